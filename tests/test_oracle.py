"""CPU tests: the oracle against the reference's own test data (golden fixtures) and against
independent solutions.  No GPU needed."""
import json
import os

import numpy as np
import pytest

import oracle as O
from blf import problems as P
from dense_qp import certify

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _g(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        return json.load(f)


# ---- ForwardEuler<LinearTimeInvariantSystem> (IntegratorTest.cpp:27-75) ----------------------
def test_integrator_lti_reference_test():
    g = _g("integrator_lti")
    cps = {c[0]: np.array(c[1:]) for c in g["checkpoints"]}
    x = np.zeros(2)
    for i in range(g["calls"]):
        t = g["dT"] * i
        closed = np.array([1 - np.exp(-t) * (np.cos(t) + np.sin(t)), 2 * np.exp(-t) * np.sin(t)])
        assert np.linalg.norm(x - closed) <= 1e-3 * min(np.linalg.norm(x), np.linalg.norm(closed))
        if i in cps:
            np.testing.assert_array_equal(x, cps[i])
        st, x, n = O.lti_euler_integrate(g["A"], g["B"], g["u"], x, 0.0, g["dT"], g["dT"])
        assert st == 0 and n == 1
    np.testing.assert_array_equal(x, g["final"])


def test_integrator_step_schedule_quirks():
    ramp = dict(A=[[0.0]], B=[[1.0]], u=[1.0])
    # dT=0.01, T=0.05: 5 steps, the last spans 2 dT from the stale time -> ends at 0.06
    st, x, n = O.lti_euler_integrate(ramp["A"], ramp["B"], ramp["u"], [0.0], 0.0, 0.05, 0.01)
    assert st == 0 and n == 5 and abs(x[0] - 0.06) < 1e-15
    # t0=1, T=1.04: ceil(4.000000000000004) = 5 steps
    st, x, n = O.lti_euler_integrate(ramp["A"], ramp["B"], ramp["u"], [0.0], 1.0, 1.04, 0.01)
    assert st == 0 and n == 5
    # errors: t0 > T and dT <= 0 are rejected; t0 == T is refused (the reference never returns)
    assert O.lti_euler_integrate(ramp["A"], ramp["B"], ramp["u"], [0.0], 1.0, 0.5, 0.1)[0] == 4
    assert O.lti_euler_integrate(ramp["A"], ramp["B"], ramp["u"], [0.0], 0.0, 1.0, 0.0)[0] == 4
    assert O.lti_euler_integrate(ramp["A"], ramp["B"], ramp["u"], [0.0], 1.0, 1.0, 0.1)[0] == 5


def test_integrator_lti_large_system_is_euler():
    """n, m above 8 (any size, as LinearTimeInvariantSystem.cpp:13-38): the same step, pinned
    against a plain numpy Euler loop of the reference's schedule (to rounding); empty sizes are
    refused."""
    rng = np.random.default_rng(5)
    n, m = 40, 7
    A = rng.uniform(-1, 1, (n, n)) / n
    B = rng.uniform(-1, 1, (n, m))
    u = rng.uniform(-1, 1, m)
    x0 = rng.uniform(-1, 1, n)
    st, x, steps = O.lti_euler_integrate(A, B, u, x0, 0.0, 0.093, 0.01)
    assert st == 0 and steps == 10
    xr = x0.copy()
    for h in [0.01] * 9 + [0.093 - 0.08]:   # the stale last step of FixedStepIntegrator.tpp:63-70
        xr = xr + (A @ xr + B @ u) * h
    np.testing.assert_allclose(x, xr, rtol=1e-12, atol=1e-13)
    n = 700
    A = rng.uniform(-1, 1, (n, n)) / n
    B = rng.uniform(-1, 1, (n, 2))
    x0 = rng.uniform(-1, 1, n)
    st, x, steps = O.lti_euler_integrate(A, B, [0.5, -0.25], x0, 0.0, 0.025, 0.01)
    assert st == 0 and steps == 3
    xr = x0.copy()
    for h in [0.01, 0.01, 0.025 - 0.01]:
        xr = xr + (A @ xr + B @ np.array([0.5, -0.25])) * h
    np.testing.assert_allclose(x, xr, rtol=1e-12, atol=1e-13)
    assert O.lti_euler_integrate(np.zeros((0, 0)), np.zeros((0, 1)), [1.0], np.zeros(0), 0.0, 1.0, 0.1)[0] == 1


def test_dcm_rollout_is_the_lti_step():
    rng = np.random.default_rng(0)
    N = 40
    om = rng.uniform(4, 4.5, N)
    r = rng.normal(0, 0.1, (N, 2))
    xi = O.dcm_euler_rollout([0.01, -0.02], om, r, 0.02)
    x = np.array([0.01, -0.02])
    for k in range(N):   # one integrate(0, dt) of the LTI system A = w I, B = -w I per knot
        st, x, _ = O.lti_euler_integrate(om[k] * np.eye(2), -om[k] * np.eye(2), r[k], x, 0.0,
                                         0.02, 0.02)
        np.testing.assert_array_equal(x, xi[k + 1])


# ---- ContactPhaseList / ContactList ------------------------------------------------------------
def test_contact_phases_reference_fixture():
    g = _g("contact_phases")
    names = sorted(g["lists"])          # std::map<std::string, ContactList> order
    lists = [g["lists"][n] for n in names]
    begin, end, active = O.contact_phases(lists)
    assert len(begin) == len(g["phases"]) == 8
    for p, (b0, e0, act) in enumerate(g["phases"]):
        assert begin[p] == b0 and end[p] == e0
        want = {names.index(k): v for k, v in act.items()}
        got = {l: int(c) for l, c in enumerate(active[p]) if c >= 0}
        assert got == want


def test_contact_phase_quirk_next_deactivation():
    # ContactPhaseList.cpp:60 compares the NEXT deactivation with the next activation: a
    # coincident deactivation/activation yields a zero-length phase
    begin, end, active = O.contact_phases([[(0.0, 1.0)], [(1.0, 2.0)]])
    assert list(zip(begin, end)) == [(0.0, 1.0), (1.0, 1.0), (1.0, 2.0)]


def test_present_contact_reference_fixture():
    g = _g("contact_list")
    acts = np.array([c[0] for c in g["contacts"]])
    for t, want in g["present"]:
        assert O.present_index(acts, t) == want


def test_generator_phases_match_oracle():
    for F, N in ((4, 50), (6, 100), (8, 130)):
        sched = P.contact_schedule(F, N)
        dt = 0.02
        mine = P.phases_from_schedule(sched, dt)
        lists = [[(a * dt, d * dt) for a, d, _ in sched[f]] for f in ("left", "right")]
        begin, end, active = O.contact_phases(lists)
        assert len(mine) == len(begin)
        for (b0, e0, act), bo, eo, ao in zip(mine, begin, end, active):
            assert b0 == bo and e0 == eo
            assert act == {l: int(c) for l, c in enumerate(ao) if c >= 0}


# ---- ConvexHullHelper (2-D) ------------------------------------------------------------------
def test_hull_matches_qhull_fixture():
    for c in _g("hull2d")["cases"]:
        pts = np.array(c["points"])
        A, b, m = O.hull2d_hrep(pts, 16)
        assert m == c["nfacets"]
        mine = np.array(sorted(map(tuple, np.c_[A[:m], b[:m]])))
        ref = np.array(sorted(map(tuple, np.c_[np.array(c["A"]), np.array(c["b"])])))
        np.testing.assert_allclose(mine, ref, atol=1e-12)
        # ConvexHullHelperTest.cpp:53-62 idea: every input point belongs (up to the rounding of
        # b = n.v), a far point does not
        assert (pts @ A[:m].T - b[:m] <= 1e-15).all()
        assert not O.hull2d_contains(A, b, m, pts.mean(0) + 10.0)
        assert O.hull2d_contains(A, b, m, pts.mean(0))


# ---- ConvexHullHelper (3-D) ------------------------------------------------------------------
def _same_planes(A, b, Ar, br, tol=1e-9):
    """Every plane of one set within tol of some plane of the other, both ways."""
    X, Y = np.c_[A, b], np.c_[Ar, br]
    d = np.abs(X[:, None, :] - Y[None, :, :]).max(axis=2)
    return (d.min(axis=1) <= tol).all() and (d.min(axis=0) <= tol).all()


def test_hull3d_matches_qhull_fixture():
    """orc_hull3d_hrep against scipy's Qhull ("Qt"): the same planes (Qhull splits a flat face into
    triangles that share one plane; here it is one row), every input point inside exactly."""
    for c in _g("hull3d")["cases"]:
        pts = np.array(c["points"])
        A, b, m = O.hull3d_hrep(pts, 64)
        Ar, br = np.array(c["A"]), np.array(c["b"])
        assert m >= 4 and m <= len(Ar)
        assert _same_planes(A[:m], b[:m], Ar, br)
        nd = (pts[:, None, 0] * A[None, :m, 0] + pts[:, None, 1] * A[None, :m, 1]) + \
            pts[:, None, 2] * A[None, :m, 2]            # the oracle's order (b = max n . p)
        assert (nd <= b[:m]).all()
        assert all(O.halfspace_contains(A[:m], b[:m], m, q) for q in pts)
        assert not O.halfspace_contains(A[:m], b[:m], m, pts.mean(0) + 10.0)
        np.testing.assert_allclose(np.linalg.norm(A[:m], axis=1), 1.0, atol=1e-14)
    # the reference test's points and outside point (ConvexHullHelperTest.cpp:15-63)
    r = _g("hull3d_reference")
    A, b, m = O.hull3d_hrep(np.array(r["points"]), 64)
    assert all(O.halfspace_contains(A[:m], b[:m], m, q) for q in r["points"])
    assert not O.halfspace_contains(A[:m], b[:m], m, r["outside"])


def test_hull3d_degenerate():
    sq = np.array([[0.0, 0, 0.5], [1, 0, 0.5], [0, 1, 0.5], [1, 1, 0.5]])
    assert O.hull3d_hrep(sq, 64)[2] == -1                       # flat
    assert O.hull3d_hrep(sq[:3], 64)[2] == -1                   # fewer than 4 points
    rng = np.random.default_rng(2)
    sph = rng.normal(size=(16, 3))
    sph /= np.linalg.norm(sph, axis=1, keepdims=True)
    assert O.hull3d_hrep(sph, 8)[2] == -1                       # 28 planes > 8 slots
    A, b, m = O.hull3d_hrep(np.r_[sph[:6], sph[:6]], 64)        # duplicated points
    A1, b1, m1 = O.hull3d_hrep(sph[:6], 64)
    assert m == m1 and _same_planes(A[:m], b[:m], A1[:m1], b1[:m1])


def test_hull_padding_and_degenerate():
    A, b, m = O.hull2d_hrep(np.array([[0.0, 0], [1, 1], [2, 2]]), 8)   # collinear
    assert m == -1 and not A.any() and not b.any()
    A, b, m = O.hull2d_hrep(np.array([[np.cos(a), np.sin(a)] for a in np.linspace(0, 6, 12)]), 8)
    assert m == -1   # needs 12 rows > 8 slots
    A, b, m = O.hull2d_hrep(np.array([[0.0, 0], [1, 0], [0, 1], [1, 0], [0, 0]]), 8)  # duplicates
    assert m == 3


# ---- QuinticSpline --------------------------------------------------------------------------
def test_quintic_coefficients_match_sympy():
    for c in _g("quintic")["cases"]:
        kt = np.array([0.0, c["T"]])
        kp = np.array([[[c["p0"]], [c["v0"]], [c["a0"]]], [[c["p1"]], [c["v1"]], [c["a1"]]]])
        co = O.quintic_fit(kt, kp)[0, 0]
        np.testing.assert_allclose(co, c["coeffs"], rtol=1e-10, atol=1e-10)
        pva, idx = O.quintic_eval(kt, O.quintic_fit(kt, kp), np.array([0.0, c["T"]]))
        np.testing.assert_allclose(pva[0, :, 0], [c["p0"], c["v0"], c["a0"]], atol=1e-12)
        np.testing.assert_allclose(pva[1, :, 0], [c["p1"], c["v1"], c["a1"]], atol=1e-9)
        assert list(idx) == [0, 1]


# ---- DCM-MPC QP -----------------------------------------------------------------------------
@pytest.fixture(scope="module")
def qp_batch():
    return O.assemble_constraints(P.make_batch(12, horizon=100, n_footsteps=6, seed=77))


@pytest.mark.parametrize("tol_polish,bar", [(3e-4, 1e-12), (1e-6, 1e-12), (0.0, 1e-9)])
def test_dcm_mpc_oracle_against_dense_certificate(qp_batch, tol_polish, bar):
    """Default: the certified active-set polish (most problems from the active-set start, with
    no IPM iteration), exact to rounding.  tol_polish = 0: the interior point method alone, within
    north_star's 1e-9."""
    worst = 0.0
    prm = O.default_params(100, tol_polish=tol_polish)
    for i in range(qp_batch["omega"].shape[0]):
        st, xi, vrp, it = O.dcm_mpc_solve(qp_batch, prm, index=i)
        assert st == 0 and 0 <= it <= 30 and (tol_polish > 0 or it >= 3)
        xi_d, r_d = certify(qp_batch, i, xi, vrp)
        worst = max(worst, np.abs(xi - xi_d).max(), np.abs(vrp - r_d).max())
    assert worst < bar, worst


def test_dcm_mpc_polish_certifies_and_saves_iterations():
    """The polish is accepted on every problem of a larger batch, matches the dense optimum to
    1e-12 and needs fewer IPM iterations than the interior point method alone."""
    prob = O.assemble_constraints(P.make_batch(96, horizon=100, n_footsteps=6, seed=78))
    pol = np.zeros(96, np.int32)
    st, xi, vrp, it, lam = O.dcm_mpc_solve_batch_warm(prob, threads=8, polished=pol)
    st0, _, _, it0, _ = O.dcm_mpc_solve_batch_warm(prob, params=O.default_params(100, tol_polish=0.0),
                                                   threads=8)
    assert (st == 0).all() and (st0 == 0).all() and pol.all()
    assert it.mean() < 0.7 * it0.mean(), (it.mean(), it0.mean())
    for i in range(0, 96, 12):
        xd, rd = certify(prob, i, xi[i], vrp[i])
        assert np.abs(xd - xi[i]).max() < 1e-12 and np.abs(rd - vrp[i]).max() < 1e-12
    # the polished multipliers: >= 0, zero off the active facets, complementary to the slacks
    M = lam.shape[2]
    used = np.arange(M)[None, None, :] < prob["nfacets"][:, :, None]
    slack = prob["b"] - np.einsum("bkij,bkj->bki", prob["A"], vrp)
    assert (lam[used] >= 0).all() and (lam[~used] == 0).all()
    assert (np.abs(slack * lam)[used]).max() < 1e-12


def test_dcm_mpc_polish_rejects_a_wrong_active_set():
    """Rejected polishes leave the IPM iterate untouched: with tol_polish huge a polish runs at the
    top of every iteration, whatever the active set looks like, and the solve still ends at the
    certified optimum."""
    prob = O.assemble_constraints(P.make_batch(16, horizon=60, n_footsteps=4, seed=80))
    pol = np.zeros(16, np.int32)
    st, xi, vrp, it, _ = O.dcm_mpc_solve_batch_warm(prob, params=O.default_params(60, tol_polish=1e30),
                                                    threads=4, polished=pol)
    assert (st == 0).all() and pol.all()
    for i in range(0, 16, 5):
        xd, rd = certify(prob, i, xi[i], vrp[i])
        assert np.abs(rd - vrp[i]).max() < 1e-12


def test_dcm_mpc_unconstrained_is_lq_optimum():
    prob = O.assemble_constraints(P.make_batch(2, horizon=30, n_footsteps=4, seed=1))
    prob["nfacets"][:] = 0
    st, xi, vrp, it = O.dcm_mpc_solve(prob, index=0)
    assert st == 0 and it == 0     # the LQ warm start already is the optimum of an equality-only QP
    xi_d, r_d = certify(prob, 0, xi, vrp)
    assert np.abs(xi - xi_d).max() < 1e-10 and np.abs(vrp - r_d).max() < 1e-10


def test_dcm_mpc_bad_facets_and_batch_driver(qp_batch):
    prob = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in qp_batch.items()}
    prob["nfacets"][3, 7] = 9
    st, xi, vrp, it = O.dcm_mpc_solve_batch(prob, threads=3)
    assert st[3] == 3 and it[3] == 0
    np.testing.assert_array_equal(vrp[3], prob["vrp_ref"][3])
    assert (np.delete(st, 3) == 0).all()
    # the threaded driver gives the same bits as the single-problem call
    for i in (0, 5, 11):
        s1, x1, r1, i1 = O.dcm_mpc_solve(prob, index=i)
        np.testing.assert_array_equal(x1, xi[i])
        np.testing.assert_array_equal(r1, vrp[i])


def test_wave_tree_sum_order():
    rng = np.random.default_rng(3)
    for n in (1, 5, 64, 100, 128, 300):
        c = rng.uniform(0, 1, n) * 10.0 ** rng.integers(-8, 8, n)
        ref = 0.0
        for w in range(0, n, 64):
            v = np.zeros(64)
            blk = c[w:w + 64]
            v[:len(blk)] = blk
            for off in (1, 2, 4, 8, 16, 32):   # the device butterfly order (DPP, permlane)
                v = v + v[np.arange(64) ^ off]
            ref = v[0] if w == 0 else ref + v[0]
        assert O.wave_tree_sum(c) == ref


def test_dcm_mpc_polish_refuses_degenerate_active_sets():
    """Duplicated facet rows make two parallel facets active at once, and a third copy makes three:
    the polish's vertex solve is singular or over-determined there, so the certificate refuses
    (pc > 2, or parallel active normals) and the interior point method finishes alone, at the
    same optimum as the problem without the copies."""
    prob = O.assemble_constraints(P.make_batch(8, horizon=40, n_footsteps=4, seed=81))
    st0, xi0, vrp0, it0, _ = O.dcm_mpc_solve_batch_warm(prob, threads=4)
    dup = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in prob.items()}
    for q in range(8):
        for k in range(40):
            m = dup["nfacets"][q, k]
            c = min(2, 8 - m)           # repeat the first facet (up to twice)
            dup["A"][q, k, m:m + c] = dup["A"][q, k, 0]
            dup["b"][q, k, m:m + c] = dup["b"][q, k, 0]
            dup["nfacets"][q, k] = m + c
    pol = np.zeros(8, np.int32)
    st, xi, vrp, it, _ = O.dcm_mpc_solve_batch_warm(dup, threads=4, polished=pol)
    assert (st == 0).all() and (st0 == 0).all()
    assert not pol.all()   # the refusal path ran
    # wherever a duplicated facet is active the polish cannot certify; the IPM's own optimum agrees
    for q in range(8):
        if not pol[q]:
            assert np.abs(vrp[q] - vrp0[q]).max() < 1e-6
        else:
            np.testing.assert_allclose(vrp[q], vrp0[q], atol=1e-12)



def test_dcm_mpc_active_set_start_solves_most_problems_without_iterations():
    """The active-set start (polish from the facets the LQ optimum violates, up to 6 drop/add
    passes) certifies nearly every problem before the first IPM iteration; the rest fall back to
    the interior point method and end polished too."""
    prob = O.assemble_constraints(P.make_batch(256, horizon=100, n_footsteps=6, seed=83))
    pol = np.zeros(256, np.int32)
    st, xi, vrp, it, _ = O.dcm_mpc_solve_batch_warm(prob, threads=8, polished=pol)
    assert (st == 0).all() and pol.all()
    assert (it == 0).mean() >= 0.95, np.bincount(it)
    for i in range(0, 256, 32):
        xd, rd = certify(prob, i, xi[i], vrp[i])
        assert np.abs(rd - vrp[i]).max() < 1e-12 and np.abs(xd - xi[i]).max() < 1e-12


def test_oracle_batch_drivers_match_single_item_calls():
    """The threaded C batch drivers (bench.py CPU baselines) return exactly what the per-item
    entry points return."""
    import numpy as np
    from blf import problems as P
    import closed_loop as CL
    prob = P.make_batch(16, horizon=40, n_footsteps=4, seed=9)
    B, Pn, C = prob["phase_corners"].shape[:3]
    A, b, nf = O.hull2d_hrep_batch(prob["phase_corners"].reshape(B * Pn, C, 2),
                                   prob["phase_ncorners"].reshape(B * Pn), 8, threads=3)
    tab = CL.phase_table(prob)
    np.testing.assert_array_equal(A.reshape(B, Pn, 8, 2), tab["phase_A"])
    np.testing.assert_array_equal(b.reshape(B, Pn, 8), tab["phase_b"])
    np.testing.assert_array_equal(nf.reshape(B, Pn), tab["phase_nf"])
    w1 = O.dcm_phase_expand(tab, 3, prob["dt"], 40)
    w2 = O.dcm_phase_expand_batch(tab, 3, prob["dt"], 40, threads=3)
    for k in w1:
        np.testing.assert_array_equal(w1[k], w2[k])
    kt, kp, tq = P.swing_splines(prob, queries=8)
    co, pva, idx = O.quintic_batch(kt, kp, tq, threads=3)
    for s in (0, kt.shape[0] - 1):
        c1 = O.quintic_fit(kt[s], kp[s])
        p1, i1 = O.quintic_eval(kt[s], c1, tq[s])
        np.testing.assert_array_equal(co[s], c1)
        np.testing.assert_array_equal(pva[s], p1)
        np.testing.assert_array_equal(idx[s], i1)


def _hull_is_tight(pts, A, b, m, tol):
    """(A, b) of m facets is the convex hull of pts up to tol: every point satisfies every facet
    (a . p - b <= tol) and every facet touches some point (min_p b - a . p <= tol)."""
    if m < 0:
        return False
    g = pts @ A[:m].T - b[:m]            # [P, m]
    return bool(g.max() <= tol and (-g).min(axis=0).max() <= tol)


def test_hull2d_all_triples_vs_andrew_degenerate():
    """up to 8 finite points the device chains the hull by the all-triples rule, which
    is Andrew's monotone chain only in exact arithmetic.  On near-collinear, duplicate-heavy and
    tiny-scale point sets both oracle paths (the all-triples rule, and Andrew's chain forced) must
    give the convex hull up to rounding: every point inside both H-reps and every facet tight, at
    1e-12 of the set's scale.  Where the two differ in facet count (a vertex within rounding of
    collinear) the count is reported, bounded, and both are still the hull."""
    rng = np.random.default_rng(7)
    differ = 0
    cases = 0
    for kind in ("near_collinear", "duplicates", "tiny", "grid", "foot_union"):
        for _ in range(3000):
            n = int(rng.integers(3, 9))
            if kind == "near_collinear":
                t = rng.uniform(-1, 1, n)
                pts = np.stack([t, 0.3 * t + rng.normal(0, 1e-13, n)], -1)
                pts[0] += [0.0, 1e-3 * rng.choice([-1, 1])]      # one point off the line
            elif kind == "duplicates":
                base = rng.uniform(-1, 1, (max(2, n // 2), 2))
                pts = base[rng.integers(0, base.shape[0], n)]
                pts[: min(3, n)] = rng.uniform(-1, 1, (min(3, n), 2))
            elif kind == "tiny":
                pts = 1e-9 * rng.uniform(-1, 1, (n, 2)) + rng.uniform(-1, 1, 2)
            elif kind == "grid":
                pts = np.round(rng.uniform(-1, 1, (n, 2)) * 4) / 4
            else:   # two slightly rotated feet (the workloads' double support), 8 corners
                P = __import__("blf.problems", fromlist=["x"])
                pose = np.array([[0.0, 0.1, rng.normal(0, 1e-3)], [rng.normal(0, 1e-6), -0.1, rng.normal(0, 1e-3)]])
                pts = P.rectangle_corners(pose).reshape(8, 2)
            scale = max(1.0, np.abs(pts).max())
            tol = 1e-12 * scale
            O.hull2d_force_andrew(False)
            A1, b1, m1 = O.hull2d_hrep(pts)
            O.hull2d_force_andrew(True)
            A2, b2, m2 = O.hull2d_hrep(pts)
            O.hull2d_force_andrew(False)
            cases += 1
            if m1 == -1 and m2 == -1:
                continue   # degenerate (all points collinear): both refuse alike
            assert (m1 == -1) == (m2 == -1), (kind, pts, m1, m2)
            span = np.ptp(pts, axis=0).max()
            if m1 > 0 and span > 1e3 * tol:
                assert _hull_is_tight(pts, A1, b1, m1, tol), (kind, pts)
                assert _hull_is_tight(pts, A2, b2, m2, tol), (kind, pts)
            if m1 != m2 or not np.array_equal(b1, b2):
                differ += 1
    assert differ <= 0.02 * cases, (differ, cases)
