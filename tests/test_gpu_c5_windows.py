"""The config-5 windows of uncapturable DCM states on the device (tests/test_c5_windows.py has the
oracle's certificates): the warm solve the closed loop runs and a cold solve of every window of
tests/golden/c5_failed_windows_r03.npz (the 68 windows that ended at the iteration cap in round 3),
c5_hard_windows.npz (the 128 that need the most interior point iterations) and c5_pushed_windows.npz
(the 100 pushed-robot windows the round-5 solver ended unsolved; round 6), through the C
ABI, against the oracle bit for bit (status, iterations, xi, VRPs, multipliers), every one
certified (status 0, polished)."""
import os

import numpy as np
import pytest
import torch

from blf import native

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KEYS = ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")


def _load(name):
    d = dict(np.load(os.path.join(GOLDEN, name)))
    return {k: d[k] for k in KEYS}, d


@pytest.mark.parametrize("name", ["c5_failed_windows_r03.npz", "c5_hard_windows.npz", "c5_pushed_windows.npz"])
def test_c5_windows_warm_bitwise(handle, oracle, name):
    prob, d = _load(name)
    B, N = prob["omega"].shape
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in prob.items()}
    prm = native.default_params(N, tol_polish=1e-4)
    warm = dict(vrp=torch.from_numpy(d["vrp_ws"]).cuda(), lam=torch.from_numpy(d["lam_ws"]).cuda(),
                shift=1, floor=1e-3, status=torch.from_numpy(d["prev_status"]).cuda())
    out = handle.dcm_mpc_solve(dev, prm, warm=warm, lambda_out=True)
    torch.cuda.synchronize()
    st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(
        prob, vrp_ws=d["vrp_ws"], lam_ws=d["lam_ws"], shift=1, floor=1e-3,
        params=oracle.default_params(N, tol_polish=1e-4), prev_status=d["prev_status"], threads=8)
    assert (st == 0).all()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), st)
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), it)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp)
    np.testing.assert_array_equal(out["lam"].cpu().numpy(), lam)
    assert out["polished"].cpu().numpy().all()


@pytest.mark.parametrize("name", ["c5_failed_windows_r03.npz", "c5_hard_windows.npz", "c5_pushed_windows.npz"])
def test_c5_windows_cold_bitwise(handle, oracle, name):
    prob, _ = _load(name)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in prob.items()}
    out = handle.dcm_mpc_solve(dev)
    torch.cuda.synchronize()
    st, xi, vrp, it = oracle.dcm_mpc_solve_batch(prob, threads=8)
    assert (st == 0).all()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), st)
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), it)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp)


def test_c5_device_window_r05_bitwise(handle, oracle):
    """tests/golden/c5_device_windows_r05.npz: the window of the device's own c5 trajectory (round 5,
    robot 13356 at period 22 of rank 0's shard, tools/capture_c5_failures.py) whose warm start
    needed 92 interior point iterations -- past the default cap of 50.  The warm kernel's passes do
    not certify it, so it is solved again from a cold start (BLF_WARM_RETRY) and stage 2 starts cold
    (kPendingCold): 31 iterations in round 5, 22 with the round-6 polish rules.  Device and oracle
    bit for bit, certified."""
    prob, d = _load("c5_device_windows_r05.npz")
    B, N = prob["omega"].shape
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in prob.items()}
    prm = native.default_params(N, tol_polish=1e-4, max_iter=100)
    warm = dict(vrp=torch.from_numpy(d["vrp_ws"]).cuda(), lam=torch.from_numpy(d["lam_ws"]).cuda(),
                shift=1, floor=1e-3, status=torch.from_numpy(d["prev_status"]).cuda())
    out = handle.dcm_mpc_solve(dev, prm, warm=warm, lambda_out=True)
    torch.cuda.synchronize()
    st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(
        prob, vrp_ws=d["vrp_ws"], lam_ws=d["lam_ws"], shift=1, floor=1e-3,
        params=oracle.default_params(N, tol_polish=1e-4, max_iter=100), prev_status=d["prev_status"],
        threads=1, device_batch=16384)
    assert (st == 0).all() and (it == 22).all()
    for k, ref in (("status", st), ("iters", it), ("xi", xi), ("vrp", vrp), ("lam", lam)):
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref, err_msg=k)
    assert out["polished"].cpu().numpy().all()
