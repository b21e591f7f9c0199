"""Edge cases of the LDS slab staging (csrc/slab.h) in the streaming kernels, bit-exact against
the oracle: partial workgroup tiles, odd row lengths, buffers that are only 8-B aligned (the
16-B vector paths fall back to scalar ones), the largest hull sizes (dynamic LDS above 64 KB),
spline dimensions 1..3, and joint counts 0 / odd."""
import numpy as np
import pytest
import torch

from blf import native

pytestmark = pytest.mark.gpu


def _d(a, dtype=torch.float64, misalign=False):
    """Device copy of `a`; with misalign=True its data pointer is 8 B past a 16-B boundary."""
    a = np.ascontiguousarray(a)
    t = torch.as_tensor(a, dtype=dtype)
    if not misalign:
        return t.cuda()
    buf = torch.empty(t.numel() + 1, dtype=dtype, device="cuda")
    out = buf[1:].view(t.shape)
    out.copy_(t.cuda())
    assert out.data_ptr() % 16 == 8
    return out


def _out_like(shape, misalign):
    return _d(np.zeros(shape), misalign=misalign)


@pytest.mark.parametrize("B,N,misalign", [(1, 100, False), (65, 100, False), (64, 7, False),
                                          (200, 99, False), (130, 16, True), (64, 33, True),
                                          (129, 100, True), (9, 128, False), (17, 130, False),
                                          (70, 160, False), (70, 161, False), (65, 200, True),
                                          (3, 1, False)])
def test_rollout_tiles_and_alignment(handle, oracle, B, N, misalign):
    rng = np.random.default_rng(B + N)
    xi0 = rng.normal(size=(B, 2))
    om = rng.uniform(2.5, 4.0, (B, N))
    vrp = rng.normal(size=(B, N, 2)) * 0.1
    out = _out_like((B, N + 1, 2), misalign)
    handle.dcm_euler_rollout(_d(xi0, misalign=misalign), _d(om, misalign=misalign),
                             _d(vrp, misalign=misalign), 0.02, out=out)
    got = out.cpu().numpy()
    for i in range(B):   # horizons <= 160: whole-row tiles of 8 problems; longer: knot chunks
        np.testing.assert_array_equal(got[i], oracle.dcm_euler_rollout(xi0[i], om[i], vrp[i], 0.02))


def _polygons(B, P_, seed):
    rng = np.random.default_rng(seed)
    pts = np.zeros((B, P_, 2))
    npts = rng.integers(3, P_ + 1, B).astype(np.int32)
    for i in range(B):
        n = npts[i]
        ang = np.sort(rng.uniform(0, 2 * np.pi, n))
        r = rng.uniform(0.5, 1.0, n)
        p = np.c_[r * np.cos(ang), r * np.sin(ang)] + rng.normal(size=2)
        rng.shuffle(p)
        pts[i, :n] = p
    npts[::11] = 2            # degenerate -> nfacets = -1
    return pts, npts


@pytest.mark.parametrize("B,P_,M", [(1, 4, 4), (77, 8, 8), (200, 16, 32), (130, 5, 3),
                                    (64, 16, 16)])
def test_hull2d_sizes_and_tiles(handle, oracle, B, P_, M):
    pts, npts = _polygons(B, P_, seed=B + P_ + M)
    A, b, nf = handle.hull2d_hrep(_d(pts), _d(npts, torch.int32), M)
    A, b, nf = A.cpu().numpy(), b.cpu().numpy(), nf.cpu().numpy()
    for i in range(B):
        Ao, bo, mo = oracle.hull2d_hrep(pts[i, :npts[i]], M)
        assert nf[i] == mo, i
        np.testing.assert_array_equal(A[i], Ao)
        np.testing.assert_array_equal(b[i], bo)


@pytest.mark.parametrize("D,Q,S,K1", [(1, 7, 33, 4), (2, 40, 10, 4), (3, 1, 300, 4), (3, 256, 3, 4),
                                      (3, 32, 40, 3), (2, 32, 17, 11), (3, 5, 60, 2)])
def test_quintic_eval_dims_and_tiles(handle, oracle, D, Q, S, K1):
    """Workgroups whose splines' knots and coefficients fit the LDS stage (<= 512 doubles) read
    them from there, the others from global memory; both bit-exact against the oracle."""
    rng = np.random.default_rng(D * 100 + Q + K1)
    kt = np.cumsum(rng.uniform(0.1, 0.5, (S, K1)), axis=1)
    kp = rng.normal(size=(S, K1, 3, D))
    tq = kt[:, :1] - 0.05 + (kt[:, -1:] - kt[:, :1] + 0.1) * rng.uniform(size=(S, Q))
    tq[:, 0] = kt[:, min(2, K1 - 1)]       # exactly on a knot
    coeffs = handle.quintic_fit(_d(kt), _d(kp))
    pva, idx = handle.quintic_eval(_d(kt), coeffs, _d(tq))
    cg, pg, ig = coeffs.cpu().numpy(), pva.cpu().numpy(), idx.cpu().numpy()
    for s in range(S):
        po, io = oracle.quintic_eval(kt[s], cg[s], tq[s])
        np.testing.assert_array_equal(ig[s], io)
        np.testing.assert_array_equal(pg[s], po)


def test_quintic_eval_unsorted_knots_rule(handle, oracle):
    """The forward knot search keeps the reference rule (last j with t_j <= t) for any order."""
    S, K1, Q = 5, 5, 16
    rng = np.random.default_rng(3)
    kt = rng.uniform(0, 1, (S, K1))
    co = rng.normal(size=(S, K1 - 1, 2, 6))
    tq = rng.uniform(-0.1, 1.1, (S, Q))
    pva, idx = handle.quintic_eval(_d(kt), _d(co), _d(tq))
    for s in range(S):
        po, io = oracle.quintic_eval(kt[s], co[s], tq[s])
        np.testing.assert_array_equal(idx.cpu().numpy()[s], io)
        np.testing.assert_array_equal(pva.cpu().numpy()[s], po)


@pytest.mark.parametrize("B,n,misalign", [(255, 7, False), (257, 0, False), (300, 24, True),
                                          (513, 1, True)])
def test_fbk_staging(handle, oracle, B, n, misalign):
    rng = np.random.default_rng(B + n)
    R = rng.normal(size=(B, 3, 3))
    twist, sd = rng.normal(size=(B, 6)), rng.normal(size=(B, n))
    pos, q = rng.normal(size=(B, 3)), rng.normal(size=(B, n))
    dp, dR, dq = handle.fbk_dynamics(0.01, _d(R, misalign=misalign), _d(twist, misalign=misalign),
                                     _d(sd, misalign=misalign))
    dpos, dRot, dqq = _d(pos, misalign=misalign), _d(R, misalign=misalign), _d(q, misalign=misalign)
    handle.fbk_euler_integrate(0.01, dpos, dRot, dqq, _d(twist, misalign=misalign),
                               _d(sd, misalign=misalign), 0.0, 0.035, 0.01)
    for i in sorted({0, 1, B // 2, 255 if B > 255 else B - 1, B - 1}):
        rp, rR, rq = oracle.fbk_dynamics(0.01, R[i], twist[i], sd[i])
        np.testing.assert_array_equal(dp.cpu().numpy()[i], rp)
        np.testing.assert_array_equal(dR.cpu().numpy()[i], rR)
        np.testing.assert_array_equal(dq.cpu().numpy()[i], rq)
        st, p, Rn, qn = oracle.fbk_euler_integrate(0.01, pos[i], R[i], q[i], twist[i], sd[i], 0.0,
                                                   0.035, 0.01)
        np.testing.assert_array_equal(dpos.cpu().numpy()[i], p)
        np.testing.assert_array_equal(dRot.cpu().numpy()[i], Rn)
        np.testing.assert_array_equal(dqq.cpu().numpy()[i], qn)


def test_hull2d_ties_duplicates_nonfinite(handle, oracle):
    """Sorting-network path (P <= 8) vs the insertion sort: equal x, duplicate points, collinear
    runs, and NaN / inf coordinates (those polygons take the insertion-sort path)."""
    rng = np.random.default_rng(17)
    B, P_ = 96, 8
    pts = np.round(rng.normal(size=(B, P_, 2)), 1)        # coarse grid: many equal x and y
    npts = rng.integers(3, P_ + 1, B).astype(np.int32)
    pts[::5, 1] = pts[::5, 0]                               # duplicate point
    pts[1::5, :4, 0] = 0.3                                  # equal x for four points
    pts[2::7, :5] = np.c_[np.arange(5) * 0.1, np.arange(5) * 0.2]   # collinear run
    pts[3::11, 2, 0] = np.nan
    pts[4::13, 1, 1] = np.inf
    pts[5::17, 0, 0] = -np.inf
    pts[6::19, 0] = (0.0, 1.0)                              # signed-zero tie: equal keys,
    pts[6::19, 1] = (-0.0, 1.0)                             # different bits
    A, b, nf = handle.hull2d_hrep(_d(pts), _d(npts, torch.int32), 8)
    A, b, nf = A.cpu().numpy(), b.cpu().numpy(), nf.cpu().numpy()
    for i in range(B):
        Ao, bo, mo = oracle.hull2d_hrep(pts[i, :npts[i]], 8)
        assert nf[i] == mo, i
        np.testing.assert_array_equal(A[i], Ao)
        np.testing.assert_array_equal(b[i], bo)


@pytest.mark.parametrize("B,P_,M,nonfinite", [(64, 8, 8, False), (200, 8, 8, True), (130, 5, 6, False),
                                               (33, 3, 3, True)])
def test_hull2d_register_path_misaligned(handle, oracle, B, P_, M, nonfinite):
    """Input points only 8-B aligned, partial workgroups (B = 33, 130), and waves in which one
    polygon with a NaN coordinate takes the insertion sort next to sorting-network polygons."""
    pts, npts = _polygons(B, P_, seed=B * 3 + P_)
    if nonfinite:
        pts[B // 2, 1, 0] = np.nan
    A, b, nf = handle.hull2d_hrep(_d(pts, misalign=True), _d(npts, torch.int32), M)
    A, b, nf = A.cpu().numpy(), b.cpu().numpy(), nf.cpu().numpy()
    for i in range(B):
        Ao, bo, mo = oracle.hull2d_hrep(pts[i, :npts[i]], M)
        assert nf[i] == mo, i
        np.testing.assert_array_equal(A[i], Ao)
        np.testing.assert_array_equal(b[i], bo)


@pytest.mark.parametrize("B,misalign", [(65, False), (130, True), (1, True), (64, False)])
def test_contact_eval_tiles_and_alignment(handle, oracle, B, misalign):
    """contact_eval_kernel's 64-contact LDS tiles: partial tiles, and inputs only 8-B aligned (the
    three 16-B input streams fall back to slab_load)."""
    from test_gpu_contact import contact_batch
    prm, twist, pose, null = contact_batch(B, seed=B + 7)
    out = handle.contact_model_eval(_d(prm, misalign=misalign), _d(twist, misalign=misalign),
                                    _d(pose, misalign=misalign), _d(null, misalign=misalign))
    ref = oracle.contact_eval_batch(prm, twist, pose, null)
    for name, r in zip(("wrench", "autonomous", "control", "regressor"), ref):
        np.testing.assert_array_equal(out[name].cpu().numpy(), r, err_msg=name)
