"""GPU parity of the phase-indexed solve (blf_dcm_mpc_solve_phased) with the two calls it fuses,
blf_dcm_phase_expand + blf_dcm_mpc_solve_warm, bit for bit: cold windows, a warm-started
receding horizon, problems the active-set kernel hands to the interior point method (their
window is expanded into the scratch the IPM reads), knots outside every phase, and the argument
checks.  omega is passed as the plan's omega with the window offset (a strided view, no copy)."""
import numpy as np
import pytest
import torch

from blf import native
from blf import problems as P

pytestmark = pytest.mark.gpu
OUT_KEYS = ("xi", "vrp", "status", "iters", "polished", "lam")


def _table(handle, prob):
    d = lambda k: torch.from_numpy(np.ascontiguousarray(prob[k])).cuda()
    return handle.phase_table(d("nphases"), d("phase_begin"), d("phase_end"), d("phase_corners"),
                              d("phase_ncorners"), ref=d("phase_ref"))


def _two_calls(handle, tab, s, xi0, omega_w, dt, N, warm=None):
    ex = handle.dcm_phase_expand(tab, s, dt, N)
    prob = dict(ex, xi_init=xi0, omega=omega_w.contiguous())
    return handle.dcm_mpc_solve(prob, warm=warm, lambda_out=True)


def _assert_same(a, b, what):
    for k in OUT_KEYS:
        assert torch.equal(a[k], b[k]), f"{k} differs ({what})"


@pytest.mark.parametrize("N,S,B", [(100, 12, 128), (64, 4, 40), (33, 3, 7), (128, 2, 16)])
def test_phased_cold_equals_expand_then_solve(handle, N, S, B):
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=31)
    tab = _table(handle, prob)
    omega = torch.from_numpy(prob["omega"]).cuda()          # [B, N + S]
    xi0 = torch.from_numpy(prob["xi_init"]).cuda()
    for s in sorted({0, S // 2, S}):
        got = handle.dcm_mpc_solve_phased(tab, s, xi0, omega[:, s:s + N], lambda_out=True)
        ref = _two_calls(handle, tab, s, xi0, omega[:, s:s + N], prob["dt"], N)
        torch.cuda.synchronize()
        _assert_same(got, ref, f"window {s}")


def test_phased_warm_receding_horizon(handle):
    N, S, B = 100, 24, 64
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=21)
    tab = _table(handle, prob)
    omega = torch.from_numpy(prob["omega"]).cuda()
    xg = xr = torch.from_numpy(prob["xi_init"]).cuda()
    pg = pr = None
    for s in range(S):
        wg = None if pg is None else dict(vrp=pg["vrp"], lam=pg["lam"], shift=1, floor=1e-3)
        wr = None if pr is None else dict(vrp=pr["vrp"], lam=pr["lam"], shift=1, floor=1e-3)
        got = handle.dcm_mpc_solve_phased(tab, s, xg, omega[:, s:s + N], warm=wg, lambda_out=True)
        ref = _two_calls(handle, tab, s, xr, omega[:, s:s + N], prob["dt"], N, warm=wr)
        torch.cuda.synchronize()
        _assert_same(got, ref, f"window {s}")
        assert (got["status"] == 0).all(), s
        pg, pr = got, ref
        xg, xr = got["xi"][:, 1].contiguous(), ref["xi"][:, 1].contiguous()


def test_phased_pending_problems_use_the_window_scratch(handle):
    """Initial DCMs far outside the support polygons: the active-set passes do not certify, the
    IPM's stage 2 reads the expanded window from the scratch (cold and warm)."""
    N, S, B = 100, 3, 48
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=5)
    tab = _table(handle, prob)
    omega = torch.from_numpy(prob["omega"]).cuda()
    xi0 = torch.from_numpy(prob["xi_init"]).cuda().clone()
    xi0[::2] += torch.tensor([0.35, -0.25], dtype=torch.float64, device="cuda")
    got = handle.dcm_mpc_solve_phased(tab, 0, xi0, omega[:, :N], lambda_out=True)
    ref = _two_calls(handle, tab, 0, xi0, omega[:, :N], prob["dt"], N)
    torch.cuda.synchronize()
    _assert_same(got, ref, "cold")
    assert (got["iters"] > 0).any(), "no problem reached the interior point method"
    pend = (got["iters"] > 0).nonzero().flatten()
    ex = handle.dcm_phase_expand(tab, 0, prob["dt"], N)
    win = got["window"]
    for k in ("A", "b", "nfacets", "xi_ref", "vrp_ref"):
        assert torch.equal(win[k][pend], ex[k][pend]), k
    assert torch.equal(win["omega"][pend], omega[pend, :N])
    warm = dict(vrp=got["vrp"], lam=got["lam"], shift=1, floor=1e-3)
    got2 = handle.dcm_mpc_solve_phased(tab, 1, got["xi"][:, 1].contiguous(), omega[:, 1:1 + N],
                                       warm=warm, lambda_out=True)
    ref2 = _two_calls(handle, tab, 1, ref["xi"][:, 1].contiguous(), omega[:, 1:1 + N], prob["dt"],
                      N, warm=dict(vrp=ref["vrp"], lam=ref["lam"], shift=1, floor=1e-3))
    torch.cuda.synchronize()
    _assert_same(got2, ref2, "warm")


def test_phased_knots_outside_every_phase(handle):
    N, B = 30, 6
    prob = P.make_batch(B, horizon=N, n_footsteps=4, seed=2)
    tab = _table(handle, prob)
    tab["nphases"] = torch.tensor([0, 2, -5, 99, 1, 3], dtype=torch.int32, device="cuda")
    begin = tab["phase_begin"].clone()
    begin[4, 0] = float("nan")                                 # never <= t
    tab["phase_begin"] = begin
    omega = torch.from_numpy(prob["omega"]).cuda()
    xi0 = torch.from_numpy(prob["xi_init"]).cuda()
    for start in (0, 7, 10 ** 6):
        got = handle.dcm_mpc_solve_phased(tab, start, xi0, omega, lambda_out=True)
        ref = _two_calls(handle, tab, start, xi0, omega, prob["dt"], N)
        torch.cuda.synchronize()
        _assert_same(got, ref, f"start {start}")
        if start == 10 ** 6:
            assert (got["status"] == native.QP_BAD_FACETS).all()


def test_phased_rejects_bad_arguments(handle):
    N, B = 40, 4
    prob = P.make_batch(B, horizon=N + 200, n_footsteps=4, seed=3)
    tab = _table(handle, prob)
    omega = torch.from_numpy(prob["omega"]).cuda()
    xi0 = torch.from_numpy(prob["xi_init"]).cuda()
    with pytest.raises(native.BlfError) as e:   # horizon > 128: the two calls instead
        handle.dcm_mpc_solve_phased(tab, 0, xi0, omega[:, :200])
    assert e.value.code == 1
    with pytest.raises(ValueError):   # the table's M must be the QP's
        handle.dcm_mpc_solve_phased(tab, 0, xi0, omega[:, :N],
                                    params=native.default_params(N, max_facets=6))
    with pytest.raises(native.BlfError) as e:   # tol_polish = 0: the IPM alone has no phased path
        handle.dcm_mpc_solve_phased(tab, 0, xi0, omega[:, :N],
                                    params=native.default_params(N, tol_polish=0.0))
    assert e.value.code == 1


# ---- the phased solve against the ORACLE directly (not only the GPU two-call path) ----
# Oracle side: the phase polygons' H-rep by the oracle hull (orc_hull2d_hrep, bit-equal to the
# device hull, test_gpu_kernels.py), the window by orc_dcm_phase_expand, the solve by
# orc_dcm_mpc_solve_batch_warm (cold: no warm start); device side: blf_dcm_mpc_solve_phased from
# the device-built table.  Every output bit for bit, window after window.

def _oracle_table(oracle, prob):
    B, Pn, C, _ = prob["phase_corners"].shape
    A, b, nf = oracle.hull2d_hrep_batch(prob["phase_corners"].reshape(B * Pn, C, 2),
                                        prob["phase_ncorners"].reshape(B * Pn), 8, threads=8)
    return dict(nphases=prob["nphases"], phase_begin=prob["phase_begin"],
                phase_end=prob["phase_end"], phase_A=A.reshape(B, Pn, 8, 2),
                phase_b=b.reshape(B, Pn, 8), phase_nf=nf.reshape(B, Pn), phase_ref=prob["phase_ref"])


def _oracle_window_solve(oracle, otab, prob, s, xi0, N, warm=None, tol_polish=3e-4):
    w = oracle.dcm_phase_expand_batch(otab, s, prob["dt"], N, threads=8)
    w["xi_init"] = np.ascontiguousarray(xi0)
    w["omega"] = np.ascontiguousarray(prob["omega"][:, s:s + N])
    pol = np.zeros(xi0.shape[0], dtype=np.int32)
    prm = oracle.default_params(N, tol_polish=tol_polish)
    if warm is None:
        st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w, params=prm, threads=8, polished=pol)
    else:
        st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w, warm[0], warm[1], 1, 1e-3,
                                                               params=prm, threads=8, polished=pol)
    return dict(status=st, xi=xi, vrp=vrp, iters=it, lam=lam, polished=pol)


def _assert_vs_oracle(got, ref, what):
    for k in OUT_KEYS:
        np.testing.assert_array_equal(got[k].cpu().numpy(), ref[k], err_msg=f"{k} ({what})")


@pytest.mark.parametrize("N,B", [(100, 96), (64, 40), (128, 24), (37, 16)])
def test_phased_cold_vs_oracle(handle, oracle, N, B):
    S = 9
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=77)
    tab, otab = _table(handle, prob), _oracle_table(oracle, prob)
    omega = torch.from_numpy(prob["omega"]).cuda()
    xi0 = torch.from_numpy(prob["xi_init"]).cuda()
    # windows near the plan's start, where xi_init (the plan's initial DCM) is still capturable
    for s in (0, 2, 4):
        got = handle.dcm_mpc_solve_phased(tab, s, xi0, omega[:, s:s + N], lambda_out=True)
        ref = _oracle_window_solve(oracle, otab, prob, s, prob["xi_init"], N)
        torch.cuda.synchronize()
        _assert_vs_oracle(got, ref, f"N={N} window {s}")
        assert (ref["status"] == 0).all()


def test_phased_warm_vs_oracle(handle, oracle):
    """The receding horizon as TimeVaryingDCMPlanner::advance runs it (shift 1, floor 1e-3,
    tol_polish 1e-4), each side warm-started from its own previous window."""
    N, S, B = 100, 30, 64
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=21)
    tab, otab = _table(handle, prob), _oracle_table(oracle, prob)
    omega = torch.from_numpy(prob["omega"]).cuda()
    prm = native.default_params(N)
    prm.tol_polish = 1e-4
    xg, xo = torch.from_numpy(prob["xi_init"]).cuda(), prob["xi_init"]
    pg = po = None
    for s in range(S):
        wg = None if pg is None else dict(vrp=pg["vrp"], lam=pg["lam"], shift=1, floor=1e-3)
        got = handle.dcm_mpc_solve_phased(tab, s, xg, omega[:, s:s + N], warm=wg, params=prm,
                                          lambda_out=True)
        ref = _oracle_window_solve(oracle, otab, prob, s, xo, N,
                                   warm=None if po is None else (po["vrp"], po["lam"]), tol_polish=1e-4)
        torch.cuda.synchronize()
        _assert_vs_oracle(got, ref, f"window {s}")
        assert (ref["status"] == 0).all(), s
        pg, po = got, ref
        xg, xo = got["xi"][:, 1].contiguous(), np.ascontiguousarray(ref["xi"][:, 1])


def test_phased_pending_vs_oracle(handle, oracle):
    """QPs the active-set kernel hands to the IPM (initial DCM far outside the polygons): the
    IPM's result from the window scratch equals the oracle's IPM on the oracle's window."""
    N, B = 100, 48
    prob = P.make_batch(B, horizon=N + 3, n_footsteps=8, seed=5)
    tab, otab = _table(handle, prob), _oracle_table(oracle, prob)
    omega = torch.from_numpy(prob["omega"]).cuda()
    xi0 = prob["xi_init"].copy()
    xi0[::2] += np.array([0.35, -0.25])
    got = handle.dcm_mpc_solve_phased(tab, 0, torch.from_numpy(xi0).cuda(), omega[:, :N],
                                      lambda_out=True)
    ref = _oracle_window_solve(oracle, otab, prob, 0, xi0, N)
    torch.cuda.synchronize()
    _assert_vs_oracle(got, ref, "cold, pending")
    assert (ref["iters"] > 0).any(), "no problem reached the interior point method"
