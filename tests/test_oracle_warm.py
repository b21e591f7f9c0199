"""Oracle warm start of the receding-horizon re-solve (DESIGN.md section 4,
"Warm start"): from the previous window's solution shifted by one knot, the IPM reaches the same
optimum (certified by the independent dense KKT solve of tests/dense_qp.py) in fewer iterations.
CPU only."""
import numpy as np

from blf import problems as P
import dense_qp

N, S, B = 100, 24, 64


def _receding(oracle, warm, floor=1e-2, windows=S, seed=7, tol_polish=3e-4):
    full = oracle.assemble_constraints(P.make_batch(B, horizon=N + windows, n_footsteps=8, seed=seed))
    prm = oracle.default_params(N, tol_polish=tol_polish)
    xi0, prev, rec = full["xi_init"], None, []
    for s in range(windows):
        w = P.window(full, s, N, xi0)
        if warm and prev is not None:
            st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w, prev[0], prev[1], 1, floor,
                                                                   params=prm, threads=8)
        else:
            st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(w, params=prm, threads=8)
        rec.append((w, st, xi, vrp, it, lam))
        prev = (vrp, lam)
        xi0 = np.ascontiguousarray(xi[:, 1])
    return rec


def test_warm_start_same_optimum_fewer_iterations(oracle):
    # the interior point method alone (tol_polish = 0): the warm start saves iterations
    cold = _receding(oracle, False, tol_polish=0.0)
    warm0 = _receding(oracle, True, tol_polish=0.0)
    it_c = np.mean([r[4].mean() for r in cold[1:]])
    it_w = np.mean([r[4].mean() for r in warm0[1:]])
    assert it_w < 0.8 * it_c, (it_w, it_c)
    # with the polish (default): the previous active set certifies nearly every window at once
    warm = _receding(oracle, True)
    assert np.mean([(r[4] == 0).mean() for r in warm[1:]]) >= 0.95
    for s in (1, 12, 20, S - 1):
        w, st, xi, vrp, it, lam = warm[s]
        assert (st == 0).all()
        # the warm and cold windows see the same QP only if their xi_init agree; they do up to the
        # IPM's accuracy, so certify the warm solution against its own window's dense optimum
        for i in range(0, B, 16):
            xd, rd = dense_qp.certify(w, i, xi[i], vrp[i])
            assert np.abs(rd - vrp[i]).max() < 1e-12
            assert np.abs(xd - xi[i]).max() < 1e-12


def test_warm_start_multipliers_layout(oracle):
    rec = _receding(oracle, True, windows=3)
    w, st, xi, vrp, it, lam = rec[-1]
    M = lam.shape[2]
    unused = np.arange(M)[None, None, :] >= w["nfacets"][:, :, None]
    assert (lam[unused] == 0).all()
    assert (lam[~unused] >= 0).all()
    # complementarity at the optimum: a multiplier is zero up to tolerance off the active facets
    slack = w["b"] - np.einsum("bkij,bkj->bki", w["A"], vrp)
    assert (np.minimum(slack, lam)[~unused] < 1e-6).all()


def test_warm_start_shift_past_horizon_is_cold_without_lq_step(oracle):
    """shift >= N: every knot is new to the window (cold rule), only the LQ step is skipped."""
    full = oracle.assemble_constraints(P.make_batch(16, horizon=N, n_footsteps=6, seed=9))
    st_c, xi_c, vrp_c, it_c, _ = oracle.dcm_mpc_solve_batch_warm(full, threads=4)
    junk = np.full((16, N, 2), np.nan)
    st, xi, vrp, it, _ = oracle.dcm_mpc_solve_batch_warm(full, junk, np.full((16, N, 8), np.nan),
                                                         N, 1e-2, threads=4)
    assert (st == 0).all() and (st_c == 0).all()
    assert np.abs(vrp - vrp_c).max() < 1e-7
