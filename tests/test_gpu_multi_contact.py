"""Three-contact phases on the device (VERDICT r03 "missing" 1): the reference ContactPhaseList
test's lists (tests/multi_contact.py) planned as TimeVaryingDCMPlanner::advance() plans them -
device phase table (blf_hull2d_hrep), then receding-horizon windows of blf_dcm_mpc_solve_phased,
warm-started from the previous window (shift 1, floor 1e-3, tol_polish 1e-4) - against the oracle
(orc_hull2d_hrep, orc_dcm_phase_expand, orc_dcm_mpc_solve_batch_warm) bit for bit.
"spread" poses need 9 facet slots (max_facets 16: the interior point kernel with the wide knot
records); "identity" poses are the reference test's own (one 4-facet rectangle, max_facets 8:
the active-set kernel)."""
import numpy as np
import pytest
import torch

import closed_loop as CL
import multi_contact as MC
from blf import native

pytestmark = pytest.mark.gpu

OUT_KEYS = ("status", "xi", "vrp", "iters", "lam", "polished")


@pytest.mark.parametrize("poses,M,off", [("spread", 16, 0.05), ("identity", 8, 0.04),
                                         ("identity", 16, 0.04)])
def test_three_contact_receding_horizon_vs_oracle(handle, oracle, poses, M, off):
    B, N, windows = 48, 60, 12
    plan = MC.plan(B, poses=poses, seed=11, xi_offset=off)
    otab = CL.phase_table(plan, max_facets=M)
    dev = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to("cuda", dt)
    tab = handle.phase_table(dev(plan["nphases"], torch.int32), dev(plan["phase_begin"]),
                             dev(plan["phase_end"]), dev(plan["phase_corners"]),
                             dev(plan["phase_ncorners"], torch.int32), max_facets=M,
                             ref=dev(plan["phase_ref"]))
    torch.cuda.synchronize()
    for k in ("phase_A", "phase_b", "phase_nf"):
        np.testing.assert_array_equal(tab[k].cpu().numpy(), otab[k], err_msg=k)
    if poses == "spread":
        assert otab["phase_nf"].max() > 8
    omega = dev(plan["omega"])
    prm = native.default_params(N, max_facets=M, dt=plan["dt"])
    prm.tol_polish = 1e-4
    oprm = oracle.default_params(N, max_facets=M, dt=plan["dt"], tol_polish=1e-4)
    xg, xo = dev(plan["xi_init"]), plan["xi_init"]
    pg = po = None
    for s in range(windows):
        wg = None if pg is None else dict(vrp=pg["vrp"], lam=pg["lam"], shift=1, floor=1e-3)
        got = handle.dcm_mpc_solve_phased(tab, s, xg, omega[:, s:s + N], warm=wg, params=prm,
                                          lambda_out=True)
        w = oracle.dcm_phase_expand(otab, s, plan["dt"], N)
        w.update(xi_init=np.ascontiguousarray(xo), omega=np.ascontiguousarray(plan["omega"][:, s:s + N]))
        pol = np.zeros(B, dtype=np.int32)
        st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(
            w, None if po is None else po["vrp"], None if po is None else po["lam"], 1, 1e-3,
            params=oprm, threads=8, polished=pol)
        ref = dict(status=st, xi=xi, vrp=vrp, iters=it, lam=lam, polished=pol)
        torch.cuda.synchronize()
        for k in OUT_KEYS:
            np.testing.assert_array_equal(got[k].cpu().numpy(), ref[k], err_msg=f"{k} window {s}")
        assert (st == 0).all(), s
        pg, po = got, ref
        xg, xo = got["xi"][:, 1].contiguous(), np.ascontiguousarray(xi[:, 1])


@pytest.mark.parametrize("N,B", [(50, 64), (60, 2048), (40, 96)])
def test_three_contact_cold_per_knot_vs_oracle(handle, oracle, N, B):
    """The 16-slot active-set kernels on the per-knot input (blf_dcm_mpc_solve, cold; the expanded
    window of a three-contact plan): status, solution, multipliers, polish flag and active-set
    passes bit for bit against the oracle, which runs the same active-set start for 16 slots.
    Knot pairs (N = 50, 60) and one knot per lane (N = 40), a batch past the DPP-tree limit."""
    M = 16
    plan = MC.plan(B, poses="spread", seed=5, xi_offset=0.05)
    otab = CL.phase_table(plan, max_facets=M)
    w = oracle.dcm_phase_expand(otab, 3, plan["dt"], N)
    w.update(xi_init=np.ascontiguousarray(plan["xi_init"]), omega=np.ascontiguousarray(plan["omega"][:, 3:3 + N]))
    assert w["nfacets"].max() > 8
    dev = {k: torch.from_numpy(np.ascontiguousarray(w[k])).cuda() for k in
           ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")}
    prm = native.default_params(N, max_facets=M, dt=plan["dt"])
    got = handle.dcm_mpc_solve(dev, prm, lambda_out=True)
    torch.cuda.synchronize()
    oprm = oracle.default_params(N, max_facets=M, dt=plan["dt"])
    pol = np.zeros(B, np.int32)
    pas = np.zeros(B, np.int32)
    st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w, params=oprm, threads=8, polished=pol, passes=pas,
                                                           device_batch=B)
    ref = dict(status=st, xi=xi, vrp=vrp, iters=it, lam=lam, polished=pol, passes=pas)
    for k in OUT_KEYS + ("passes",):
        np.testing.assert_array_equal(got[k].cpu().numpy(), ref[k], err_msg=k)
    assert (st == 0).all()
    assert (pas > 0).all()   # the active-set kernels ran (not the interior point kernel alone)
