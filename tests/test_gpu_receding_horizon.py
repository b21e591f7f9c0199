"""GPU parity of the warm-started receding-horizon re-solve (blf_dcm_mpc_solve_warm; SURVEY.md
8(a) A3) against the oracle's warm start (orc_dcm_mpc_solve_warm): window after window, each
side warm-started from its own previous solution, bit-equal xi, vrp, multipliers, status and
iteration counts.  The windows cross the terminal-reference jumps of the plan (s = 20, 30) where
the warm start is far from the new optimum."""
import numpy as np
import pytest
import torch

from blf import problems as P

pytestmark = pytest.mark.gpu
KEYS = ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")


def _dev(w):
    return {k: torch.from_numpy(np.ascontiguousarray(w[k])).cuda() for k in KEYS}


@pytest.mark.parametrize("horizon,batch,windows", [(100, 48, 32), (64, 24, 12), (150, 16, 6)])
def test_receding_horizon_warm_bitwise(handle, oracle, horizon, batch, windows):
    full = oracle.assemble_constraints(
        P.make_batch(batch, horizon=horizon + windows, n_footsteps=8, seed=21))
    xi0_o = xi0_g = full["xi_init"]
    prev_o = prev_g = None
    for s in range(windows):
        w_o = P.window(full, s, horizon, xi0_o)
        w_g = _dev(P.window(full, s, horizon, xi0_g))
        if prev_o is None:
            st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w_o, threads=8)
            out = handle.dcm_mpc_solve(w_g, lambda_out=True)
        else:
            st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w_o, prev_o[0], prev_o[1], 1,
                                                                   1e-2, threads=8)
            out = handle.dcm_mpc_solve(w_g, warm=dict(vrp=prev_g[0], lam=prev_g[1], shift=1,
                                                      floor=1e-2), lambda_out=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out["status"].cpu().numpy(), st)
        np.testing.assert_array_equal(out["iters"].cpu().numpy(), it)
        np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi)
        np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp)
        np.testing.assert_array_equal(out["lam"].cpu().numpy(), lam)
        assert (st == 0).all(), (s, st)
        prev_o, prev_g = (vrp, lam), (out["vrp"], out["lam"])
        xi0_o, xi0_g = np.ascontiguousarray(xi[:, 1]), out["xi"][:, 1].cpu().numpy()


@pytest.mark.parametrize("shift,floor", [(0, 1e-2), (3, 1e-3), (7, 1e-6), (200, 1e-2)])
def test_warm_shift_and_floor_bitwise(handle, oracle, shift, floor):
    """Other shifts (0: re-solve in place; >= N: all knots new) and floors."""
    B, N = 32, 100
    full = oracle.assemble_constraints(P.make_batch(B, horizon=N + 10, n_footsteps=8, seed=4))
    w0 = P.window(full, 0, N)
    st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w0, threads=8)
    w1 = P.window(full, min(shift, 10), N, np.ascontiguousarray(xi[:, min(shift, N)]))
    st1, xi1, vrp1, it1, lam1 = oracle.dcm_mpc_solve_batch_warm(w1, vrp, lam, shift, floor, threads=8)
    out = handle.dcm_mpc_solve(
        _dev(w1), warm=dict(vrp=torch.from_numpy(vrp).cuda(), lam=torch.from_numpy(lam).cuda(),
                            shift=shift, floor=floor), lambda_out=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), st1)
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), it1)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi1)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp1)
    np.testing.assert_array_equal(out["lam"].cpu().numpy(), lam1)


def test_cold_lambda_out_and_bad_facets(handle, oracle):
    """lambda_out of a cold solve (no warm start) and of a problem rejected for its facet count."""
    B, N = 8, 40
    host = oracle.assemble_constraints(P.make_batch(B, horizon=N, n_footsteps=4, seed=3))
    host["nfacets"][2, 5] = 9
    st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(host, threads=4)
    out = handle.dcm_mpc_solve(_dev(host), lambda_out=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), st)
    np.testing.assert_array_equal(out["lam"].cpu().numpy(), lam)
    assert st[2] == 3 and (lam[2] == 0).all()


def test_warm_rejects_bad_arguments(handle, oracle):
    from blf import native
    B, N = 4, 20
    host = oracle.assemble_constraints(P.make_batch(B, horizon=N, n_footsteps=4, seed=3))
    dev = _dev(host)
    out = handle.dcm_mpc_solve(dev, lambda_out=True)
    for bad in (dict(shift=-1), dict(floor=0.0), dict(floor=float("nan"))):
        kw = dict(vrp=out["vrp"].clone(), lam=out["lam"].clone(), shift=1, floor=1e-2)
        kw.update(bad)
        with pytest.raises(native.BlfError):
            handle.dcm_mpc_solve(dev, warm=kw)
    # the warm start must not alias the outputs
    with pytest.raises(native.BlfError):
        handle.dcm_mpc_solve(dev, out=out, warm=dict(vrp=out["vrp"], lam=out["lam"].clone()))


def test_failed_window_restarts_cold(handle, oracle):
    """A window whose QP failed does not seed the next window: with the previous statuses in the
    warm start (blf_dcm_mpc_warm_start.prev_status), the failed problems are solved exactly as a
    cold solve solves them, the others warm, bit for bit against the oracle's batch driver with
    the same prev_status.  The failed problems' warm start is poisoned (VRPs far outside every
    polygon, huge multipliers) to show that none of it is read."""
    from blf import native
    B, N = 24, 100
    full = oracle.assemble_constraints(P.make_batch(B, horizon=N + 2, n_footsteps=8, seed=9))
    w0 = P.window(full, 0, N)
    out0 = handle.dcm_mpc_solve(_dev(w0), lambda_out=True)
    torch.cuda.synchronize()
    assert (out0["status"] == 0).all()
    failed = torch.zeros(B, dtype=torch.bool, device="cuda")
    failed[::3] = True
    vrp_ws, lam_ws = out0["vrp"].clone(), out0["lam"].clone()
    vrp_ws[failed] = 5.0
    lam_ws[failed] = 1e6
    st_ws = torch.where(failed, native.QP_MAX_ITER, 0).to(torch.int32)
    xi1 = out0["xi"][:, 1].cpu().numpy()
    w1 = P.window(full, 1, N, xi1)
    warm = dict(vrp=vrp_ws, lam=lam_ws, shift=1, floor=1e-2, status=st_ws)
    got = handle.dcm_mpc_solve(_dev(w1), warm=warm, lambda_out=True)
    cold = handle.dcm_mpc_solve(_dev(w1), lambda_out=True)
    plain = handle.dcm_mpc_solve(_dev(w1), warm=dict(warm, status=None), lambda_out=True)
    torch.cuda.synchronize()
    for k in ("xi", "vrp", "status", "iters", "lam"):
        assert torch.equal(got[k][failed], cold[k][failed]), k          # restarted cold
        assert torch.equal(got[k][~failed], plain[k][~failed]), k       # warm as before
    assert (got["status"] == 0).all()
    st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(
        w1, vrp_ws.cpu().numpy(), lam_ws.cpu().numpy(), 1, 1e-2, threads=8,
        prev_status=st_ws.cpu().numpy())
    np.testing.assert_array_equal(got["status"].cpu().numpy(), st)
    np.testing.assert_array_equal(got["iters"].cpu().numpy(), it)
    np.testing.assert_array_equal(got["xi"].cpu().numpy(), xi)
    np.testing.assert_array_equal(got["vrp"].cpu().numpy(), vrp)
    np.testing.assert_array_equal(got["lam"].cpu().numpy(), lam)
    # the warm start's statuses must not alias the output statuses
    with pytest.raises(native.BlfError):
        handle.dcm_mpc_solve(_dev(w1), out=got, warm=dict(warm, status=got["status"]), lambda_out=True)
