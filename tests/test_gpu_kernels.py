"""GPU parity of the rollout, hull and spline kernels against the oracle (bit-exact: same
expression order, no FMA contraction on either side) and against the reference's own fixtures."""
import json
import os

import numpy as np
import pytest
import torch

from blf import native
from blf import problems as P

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _d(a, dtype=torch.float64):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dtype).cuda()


def test_lti_integrator_matches_reference_test_and_oracle(handle, oracle):
    """IntegratorTest.cpp:27-75: A=[[0,1],[-2,-2]], B=[0,2]^T, u=1, dT=1e-4, 20000 calls of
    integrate(0, dT); solution isApprox(closed form, 1e-3) before every call."""
    with open(os.path.join(GOLDEN, "integrator_lti.json")) as f:
        g = json.load(f)
    A = _d(np.array(g["A"]))
    B = _d(np.array(g["B"]))
    u = _d(np.array([[1.0]]))
    x = _d(np.zeros((1, 2)))
    dT = g["dT"]
    xo = np.zeros(2)
    checkpoints = {c[0]: np.array(c[1:]) for c in g["checkpoints"]}
    for i in range(g["calls"]):
        if i in checkpoints:
            # bit-exact vs the fixture (oracle-generated, closed-form-checked at every step)
            np.testing.assert_array_equal(x.cpu().numpy()[0], checkpoints[i])
        handle.lti_euler_integrate(A, B, u, x, 0.0, dT, dT, shared=True)
        _, xo, _ = oracle.lti_euler_integrate(g["A"], g["B"], [1.0], xo, 0.0, dT, dT)
    np.testing.assert_array_equal(x.cpu().numpy()[0], xo)
    t = dT * g["calls"]
    closed = np.array([1 - np.exp(-t) * (np.cos(t) + np.sin(t)), 2 * np.exp(-t) * np.sin(t)])
    assert np.linalg.norm(xo - closed) <= 1e-3 * min(np.linalg.norm(xo), np.linalg.norm(closed))


@pytest.mark.parametrize("t0,t1,dT", [(0.0, 0.05, 0.01), (1.0, 1.04, 0.01), (0.0, 1e-4, 1e-4),
                                      (0.3, 2.0, 0.07)])
def test_lti_integrator_step_schedule(handle, oracle, t0, t1, dT):
    rng = np.random.default_rng(0)
    B, n, m = 257, 3, 2
    A = rng.uniform(-1, 1, (B, n, n))
    Bm = rng.uniform(-1, 1, (B, n, m))
    u = rng.uniform(-1, 1, (B, m))
    x0 = rng.uniform(-1, 1, (B, n))
    x = _d(x0)
    handle.lti_euler_integrate(_d(A), _d(Bm), _d(u), x, t0, t1, dT)
    xg = x.cpu().numpy()
    for i in range(0, B, 37):
        st, xo, _ = oracle.lti_euler_integrate(A[i], Bm[i], u[i], x0[i], t0, t1, dT)
        assert st == 0
        np.testing.assert_array_equal(xg[i], xo)


@pytest.mark.parametrize("n,m,shared", [(9, 3, False), (12, 8, True), (40, 17, False), (130, 1, True),
                                        (5, 20, False)])
def test_lti_integrator_large_systems(handle, oracle, n, m, shared):
    """n or m above 8: one workgroup per system (lti_euler_wg_kernel), bit-identical to the
    oracle's step (the same left-to-right sums), per-system and shared matrices."""
    rng = np.random.default_rng(n * 100 + m)
    B = 37
    A = rng.uniform(-1, 1, (n, n) if shared else (B, n, n)) / n
    Bm = rng.uniform(-1, 1, (n, m) if shared else (B, n, m))
    u = rng.uniform(-1, 1, (B, m))
    x0 = rng.uniform(-1, 1, (B, n))
    x = _d(x0)
    handle.lti_euler_integrate(_d(A), _d(Bm), _d(u), x, 0.0, 0.093, 0.01, shared=shared)
    xg = x.cpu().numpy()
    for i in range(B):
        st, xo, steps = oracle.lti_euler_integrate(A if shared else A[i], Bm if shared else Bm[i], u[i],
                                                   x0[i], 0.0, 0.093, 0.01)
        assert st == 0 and steps == 10
        np.testing.assert_array_equal(xg[i], xo)
    dx = handle.lti_dynamics(_d(A), _d(Bm), _d(u), _d(x0), shared=shared).cpu().numpy()
    for i in range(0, B, 6):
        Ai, Bi = (A, Bm) if shared else (A[i], Bm[i])
        np.testing.assert_allclose(dx[i], Ai @ x0[i] + Bi @ u[i], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("n,m,shared,B", [(513, 1, True, 3), (600, 700, False, 2), (9, 600, True, 4),
                                          (1100, 2, True, 1)])
def test_lti_integrator_any_size(handle, oracle, n, m, shared, B):
    """Above 512 (lti_euler_big_kernel, lti_dynamics_rows_kernel; the reference takes any size,
    LinearTimeInvariantSystem.cpp:13-38): bit-identical to the oracle's left-to-right sums."""
    rng = np.random.default_rng(n + 7 * m)
    A = rng.uniform(-1, 1, (n, n) if shared else (B, n, n)) / n
    Bm = rng.uniform(-1, 1, (n, m) if shared else (B, n, m)) / m
    u = rng.uniform(-1, 1, (B, m))
    x0 = rng.uniform(-1, 1, (B, n))
    x = _d(x0)
    handle.lti_euler_integrate(_d(A), _d(Bm), _d(u), x, 0.0, 0.045, 0.01, shared=shared)
    xg = x.cpu().numpy()
    for i in range(B):
        st, xo, steps = oracle.lti_euler_integrate(A if shared else A[i], Bm if shared else Bm[i], u[i],
                                                   x0[i], 0.0, 0.045, 0.01)
        assert st == 0 and steps == 5
        np.testing.assert_array_equal(xg[i], xo)
    dx = handle.lti_dynamics(_d(A), _d(Bm), _d(u), _d(x0), shared=shared).cpu().numpy()
    for i in range(B):
        Ai, Bi = (A, Bm) if shared else (A[i], Bm[i])
        ax = np.zeros(n); bu = np.zeros(n)
        ax[:] = Ai[:, 0] * x0[i, 0]
        for c in range(1, n):
            ax = ax + Ai[:, c] * x0[i, c]
        bu[:] = Bi[:, 0] * u[i, 0]
        for c in range(1, m):
            bu = bu + Bi[:, c] * u[i, c]
        np.testing.assert_array_equal(dx[i], ax + bu)   # the same left-to-right sums, bit for bit


def test_lti_integrator_size_limit(handle):
    """Empty systems are refused by the C ABI (the adapter handles n = 0 and m = 0 itself)."""
    A = _d(np.eye(1)); x = _d(np.zeros((1, 1)))
    for n, m in [(0, 1), (1, 0)]:
        rc = native.lib().blf_lti_euler_integrate(handle._h, n, m, A.data_ptr(), A.data_ptr(), 1,
                                                  A.data_ptr(), x.data_ptr(), 1, 0.0, 1.0, 0.1, None)
        assert rc == 1
        rc = native.lib().blf_lti_dynamics(handle._h, n, m, A.data_ptr(), A.data_ptr(), 1, A.data_ptr(),
                                           x.data_ptr(), x.data_ptr(), 1, None)
        assert rc == 1


def test_lti_integrator_errors(handle):
    A = _d(np.eye(2)); B = _d(np.ones((2, 1))); u = _d(np.ones((1, 1))); x = _d(np.zeros((1, 2)))
    with pytest.raises(native.BlfError) as e:
        handle.lti_euler_integrate(A, B, u, x, 1.0, 0.5, 0.1, shared=True)
    assert e.value.code == 4
    with pytest.raises(native.BlfError) as e:
        handle.lti_euler_integrate(A, B, u, x, 0.0, 1.0, 0.0, shared=True)
    assert e.value.code == 4
    with pytest.raises(native.BlfError) as e:
        handle.lti_euler_integrate(A, B, u, x, 1.0, 1.0, 0.1, shared=True)
    assert e.value.code == 5


def test_dcm_rollout_bitwise(handle, oracle):
    prob = P.make_batch(300, horizon=100, seed=2)
    rng = np.random.default_rng(1)
    vrp = prob["vrp_ref"] + rng.normal(0, 0.01, prob["vrp_ref"].shape)
    out = handle.dcm_euler_rollout(_d(prob["xi_init"]), _d(prob["omega"]), _d(vrp), 0.02)
    og = out.cpu().numpy()
    for i in range(0, 300, 7):
        ref = oracle.dcm_euler_rollout(prob["xi_init"][i], prob["omega"][i], vrp[i], 0.02)
        np.testing.assert_array_equal(og[i], ref)


def test_hull2d_matches_oracle_and_qhull_fixture(handle, oracle):
    with open(os.path.join(GOLDEN, "hull2d.json")) as f:
        cases = json.load(f)["cases"]
    B = len(cases)
    P_ = 16
    pts = np.zeros((B, P_, 2))
    npts = np.zeros(B, dtype=np.int32)
    for i, c in enumerate(cases):
        p = np.array(c["points"])
        pts[i, :len(p)] = p
        npts[i] = len(p)
    A, b, nf = handle.hull2d_hrep(_d(pts), _d(npts, torch.int32), 8)
    A, b, nf = A.cpu().numpy(), b.cpu().numpy(), nf.cpu().numpy()
    for i, c in enumerate(cases):
        Ao, bo, mo = oracle.hull2d_hrep(pts[i, :npts[i]], 8)
        assert nf[i] == mo
        np.testing.assert_array_equal(A[i], Ao)
        np.testing.assert_array_equal(b[i], bo)
        # Qhull "Qt" fixture: same facet set (order is Qhull-internal), tol 1e-12
        if c["nfacets"] > 8:
            assert nf[i] == -1
            continue
        assert nf[i] == c["nfacets"]
        mine = sorted(map(tuple, np.round(np.c_[A[i, :nf[i]], b[i, :nf[i]]], 12)))
        ref = sorted(map(tuple, np.round(np.c_[np.array(c["A"]), np.array(c["b"])], 12)))
        np.testing.assert_allclose(np.array(mine), np.array(ref), atol=1e-12)


def _sets3d(B, P_, seed):
    """3-D point sets for hull3d_kernel: points on spheres, boxes with interior points, cubes (flat
    faces), flat sets, too few points, duplicates."""
    rng = np.random.default_rng(seed)
    pts = np.zeros((B, P_, 3))
    npts = rng.integers(4, P_ + 1, B).astype(np.int32)
    for i in range(B):
        n = npts[i]
        kind = i % 5
        if kind == 0:
            p = rng.normal(size=(n, 3))
            p /= np.linalg.norm(p, axis=1, keepdims=True)
        elif kind == 1:
            p = rng.uniform(-1.0, 2.0, (n, 3))
        elif kind == 2:
            p = np.array([[x, y, z] for x in (0.0, 1.0) for y in (0.0, 1.0) for z in (0.0, 1.0)])
            p = np.r_[p, rng.uniform(0.1, 0.9, (max(0, n - 8), 3))][:n] * rng.uniform(0.5, 2.0)
            n = npts[i] = len(p)
        elif kind == 3:
            p = np.c_[rng.uniform(size=(n, 2)), np.full(n, 0.3)]        # flat: no hull
        else:
            p = rng.normal(size=(n, 3))
            p[n // 2:] = p[:n - n // 2]                                   # duplicates
        pts[i, :n] = p + rng.normal(size=3)
    npts[5::17] = 3                                                       # too few points
    return pts, npts


@pytest.mark.parametrize("B,P_,M", [(1, 8, 32), (70, 16, 32), (130, 12, 8)])
def test_hull3d_matches_oracle(handle, oracle, B, P_, M):
    """hull3d_kernel (ConvexHullHelper on 3 x p points) bit for bit against orc_hull3d_hrep, which
    tests/test_oracle.py pins to scipy's Qhull; halfspace_contains against the oracle."""
    pts, npts = _sets3d(B, P_, seed=B + P_)
    A, b, nf = handle.hull3d_hrep(_d(pts), _d(npts, torch.int32), M)
    An, bn, nn = A.cpu().numpy(), b.cpu().numpy(), nf.cpu().numpy()
    for i in range(B):
        Ao, bo, mo = oracle.hull3d_hrep(pts[i, :npts[i]], M)
        assert nn[i] == mo, i
        np.testing.assert_array_equal(An[i], Ao)
        np.testing.assert_array_equal(bn[i], bo)
    rng = np.random.default_rng(B)
    q = pts[:, :4].mean(axis=1) + rng.normal(0, 0.6, (B, 3))
    inside = handle.halfspace_contains(A, b, nf, _d(q)).cpu().numpy()
    for i in range(B):
        assert inside[i] == oracle.halfspace_contains(An[i], bn[i], int(nn[i]), q[i])
    ok = nn >= 0
    assert ok.any() and (B == 1 or (~ok).any())
    # every input point of a valid hull is inside exactly (b = max n . p)
    for i in np.flatnonzero(ok):
        p, a = pts[i, :npts[i], None, :], An[None, i, :nn[i], :]
        nd = (p[..., 0] * a[..., 0] + p[..., 1] * a[..., 1]) + p[..., 2] * a[..., 2]
        assert (nd <= bn[i, :nn[i]]).all()


def test_halfspace_contains_2d_matches_hull2d_contains(handle):
    """The dimension-generic containment test on the planner's 2-D polygons agrees with the 2-D one."""
    rng = np.random.default_rng(5)
    prob = P.make_batch(64, horizon=7, seed=3)
    pts = prob["corners"][:, :8].reshape(-1, 8, 2)
    npts = prob["ncorners"][:, :8].reshape(-1).astype(np.int32)
    A, b, nf = handle.hull2d_hrep(_d(pts), _d(npts, torch.int32), 8)
    q = _d(pts.mean(axis=1) + rng.normal(0, 0.08, (pts.shape[0], 2)))
    np.testing.assert_array_equal(handle.halfspace_contains(A, b, nf, q).cpu().numpy(),
                                  handle.hull2d_contains(A, b, nf, q).cpu().numpy())


def test_hull2d_contains(handle, oracle):
    rng = np.random.default_rng(4)
    B = 4096
    prob = P.make_batch(B // 8, horizon=7, seed=9)
    pts = prob["corners"][:, :8].reshape(-1, 8, 2)
    npts = prob["ncorners"][:, :8].reshape(-1).astype(np.int32)
    A, b, nf = handle.hull2d_hrep(_d(pts), _d(npts, torch.int32), 8)
    q = pts.mean(axis=1) + rng.normal(0, 0.08, (pts.shape[0], 2))
    inside = handle.hull2d_contains(A, b, nf, _d(q)).cpu().numpy()
    An, bn, nn = A.cpu().numpy(), b.cpu().numpy(), nf.cpu().numpy()
    for i in range(0, pts.shape[0], 13):
        assert inside[i] == oracle.hull2d_contains(An[i], bn[i], int(nn[i]), q[i])
    # every corner belongs to its own hull up to rounding of b = n.v (ConvexHullHelperTest idea)
    assert (np.einsum("bij,bkj->bik", An, pts) - bn[:, :, None] <= 1e-15).all()


def test_quintic_fit_eval_bitwise_and_knot_rule(handle, oracle):
    prob = P.make_batch(64, horizon=100, n_footsteps=6, seed=8)
    kt, kp, tq = P.swing_splines(prob, queries=40)
    tq = tq.copy()
    tq[:, 0] -= 0.01     # before the first knot -> idx -1 (getPresentContact end())
    tq[:, -1] += 0.01    # after the last knot -> idx K
    tq[:, 5] = kt[:, 1]  # exactly on the apex knot -> that knot (`<=`)
    coeffs = handle.quintic_fit(_d(kt), _d(kp))
    pva, idx = handle.quintic_eval(_d(kt), coeffs, _d(tq))
    cg, pg, ig = coeffs.cpu().numpy(), pva.cpu().numpy(), idx.cpu().numpy()
    for s in range(0, kt.shape[0], 5):
        co = oracle.quintic_fit(kt[s], kp[s])
        np.testing.assert_array_equal(cg[s], co)
        po, io = oracle.quintic_eval(kt[s], co, tq[s])
        np.testing.assert_array_equal(ig[s], io)
        np.testing.assert_array_equal(pg[s], po)
        for j, t in enumerate(tq[s]):
            assert io[j] == oracle.present_index(kt[s], t)
    assert (ig[:, 0] == -1).all() and (ig[:, -1] == 2).all() and (ig[:, 5] == 1).all()
