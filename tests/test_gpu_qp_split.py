"""The large-batch split of the cold active-set kernel (blf_set_qp_split_batch):
the fp32 search as its own kernel at four wavefronts per SIMD, its hand-over state parked in the
output arrays, then the fp64 certification kernel.  Split and fused launches give the same bits,
and both the oracle's, for knot pairs (N = 100, 128) and one knot per lane (N = 50, at a batch
past the DPP-tree bound), with QPs handed to the IPM's stage 2 (initial DCMs far outside the
support polygons) and the multipliers requested or not."""
import numpy as np
import pytest
import torch

from blf import native
from blf import problems as P

pytestmark = pytest.mark.gpu

KEYS = ("status", "xi", "vrp", "iters", "polished", "lam")


def _dev(handle, prob):
    d = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).cuda()
         for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}
    A, b, nf = handle.assemble_constraints(torch.from_numpy(prob["corners"]).cuda(),
                                           torch.from_numpy(prob["ncorners"]).cuda())
    d.update(A=A, b=b, nfacets=nf)
    return d


@pytest.mark.parametrize("horizon,footsteps,batch", [(100, 6, 1536), (50, 4, 1280), (128, 8, 512)])
def test_split_equals_fused_and_oracle(handle, oracle, horizon, footsteps, batch):
    prob = P.make_batch(batch, horizon=horizon, n_footsteps=footsteps, seed=17)
    prob["xi_init"][::7] += np.array([0.3, -0.2])     # a few QPs go on to the interior point kernel
    dev = _dev(handle, prob)
    res = {}
    prev = native.set_qp_split_batch(-1)
    try:
        for split in (0, 1):
            native.set_qp_split_batch(1 if split else 0)
            for lam in (True, False):
                out = handle.dcm_mpc_solve(dev, lambda_out=lam)
                torch.cuda.synchronize()
                res[(split, lam)] = {k: v.cpu().numpy().copy() for k, v in out.items() if k in KEYS}
    finally:
        native.set_qp_split_batch(prev)
    host = dict(prob)
    for k in ("A", "b", "nfacets"):
        host[k] = dev[k].cpu().numpy()
    pol = np.zeros(batch, np.int32)
    st, xi, vrp, it, lamo = oracle.dcm_mpc_solve_batch_warm(
        host, params=oracle.default_params(horizon), threads=8, polished=pol, device_batch=batch)
    ref = dict(status=st, xi=xi, vrp=vrp, iters=it, polished=pol, lam=lamo)
    assert (it > 0).any(), "no QP reached the interior point kernel"
    for (split, lam), r in res.items():
        for k in KEYS:
            if k in r:
                np.testing.assert_array_equal(r[k], ref[k], err_msg=f"{k} split={split} lam={lam}")


def test_split_batch_setting_roundtrip():
    prev = native.set_qp_split_batch(-1)
    try:
        assert native.set_qp_split_batch(4096) == prev
        assert native.set_qp_split_batch(0) == 4096
        assert native.set_qp_split_batch(-1) == 0
    finally:
        native.set_qp_split_batch(prev)
