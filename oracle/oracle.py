"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
The product path (bipedal-locomotion-framework_amd/blf) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


class OrcFbModel(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("parent", _ip), ("joint_origin", _dp), ("joint_rot", _dp),
                ("joint_axis", _dp), ("link_mass", _dp), ("link_com", _dp), ("link_inertia", _dp),
                ("frame_link", _ip), ("frame_pose", _dp), ("gravity", ctypes.c_double * 3),
                ("rho", ctypes.c_double), ("joint_type", _ip)]


class OrcParams(ctypes.Structure):
    _fields_ = [("horizon", ctypes.c_int32), ("max_facets", ctypes.c_int32),
                ("max_iter", ctypes.c_int32), ("sequential", ctypes.c_int32),
                ("dt", ctypes.c_double), ("w_xi", ctypes.c_double * 2),
                ("w_vrp", ctypes.c_double * 2), ("w_terminal", ctypes.c_double * 2),
                ("tol_mu", ctypes.c_double), ("tol_primal", ctypes.c_double),
                ("tol_dual", ctypes.c_double), ("tol_polish", ctypes.c_double),
                ("single_kernel", ctypes.c_int32), ("as_tree", ctypes.c_int32)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        # BLF_ORACLE_LIB: another build of the same sources (the ASan/UBSan build of
        # `make -C oracle asan`, run by tests/test_sanitizers.py under LD_PRELOAD=libasan)
        path = os.environ.get("BLF_ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.orc_lti_euler_integrate.restype = ctypes.c_int
        L.orc_lti_euler_integrate.argtypes = [ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, _dp,
                                              ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                              ctypes.POINTER(ctypes.c_int64)]
        L.orc_dcm_euler_rollout.argtypes = [_dp, _dp, _dp, ctypes.c_int, ctypes.c_double, _dp]
        L.orc_contact_phases.restype = ctypes.c_int
        L.orc_contact_phases.argtypes = [ctypes.c_int, ctypes.c_int, _dp, _dp, _ip, ctypes.c_int,
                                         _dp, _dp, _ip]
        L.orc_present_index.restype = ctypes.c_int
        L.orc_present_index.argtypes = [_dp, ctypes.c_int, ctypes.c_double]
        L.orc_hull2d_hrep.restype = ctypes.c_int
        L.orc_hull2d_hrep.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_hull3d_hrep.argtypes = [_dp, ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_halfspace_contains.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_hullnd_hrep.argtypes = [ctypes.c_int, _dp, ctypes.c_int, ctypes.c_int, _dp, _dp]
        L.orc_hull2d_contains.restype = ctypes.c_int
        L.orc_hull2d_contains.argtypes = [_dp, _dp, ctypes.c_int, _dp]
        L.orc_quintic_fit.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, _dp]
        L.orc_quintic_eval.argtypes = [_dp, _dp, ctypes.c_int, ctypes.c_int, _dp, ctypes.c_int,
                                       _dp, _ip]
        L.orc_dcm_mpc_solve.restype = ctypes.c_int
        L.orc_dcm_mpc_solve.argtypes = [ctypes.POINTER(OrcParams), _dp, _dp, _dp, _dp, _dp, _dp,
                                        _ip, _dp, _dp, _ip]
        L.orc_dcm_mpc_solve_batch.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int64,
                                              ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _ip,
                                              _dp, _dp, _ip, _ip]
        L.orc_dcm_mpc_solve_batch_warm.argtypes = [
            ctypes.POINTER(OrcParams), ctypes.c_int64, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp,
            _ip, _dp, _dp, _ip, ctypes.c_int32, ctypes.c_double, _dp, _dp, _dp, _ip, _ip, _ip, _ip]
        L.orc_dcm_phase_expand.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp, _dp,
                                           _dp, _dp, _ip, _dp, ctypes.c_int64, ctypes.c_double,
                                           ctypes.c_int, _dp, _dp, _ip, _dp, _dp]
        L.orc_hull2d_hrep_batch.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, _dp, _ip,
                                            _dp, _dp, _ip, ctypes.c_int]
        L.orc_dcm_phase_expand_batch.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, _ip,
                                                 _dp, _dp, _dp, _dp, _ip, _dp, ctypes.c_int64,
                                                 ctypes.c_double, ctypes.c_int, _dp, _dp, _ip, _dp,
                                                 _dp, ctypes.c_int]
        L.orc_quintic_batch.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        _dp, _dp, _dp, _dp, _dp, _ip, ctypes.c_int]
        L.orc_wave_tree_sum.restype = ctypes.c_double
        L.orc_wave_tree_sum.argtypes = [_dp, ctypes.c_int]
        L.orc_contact_eval.argtypes = [_dp] * 8
        L.orc_contact_point.argtypes = [_dp, _dp, _dp, _dp, ctypes.c_double, ctypes.c_double,
                                        _dp, _dp]
        L.orc_fbk_dynamics.argtypes = [ctypes.c_int, ctypes.c_double, _dp, _dp, _dp, _dp, _dp,
                                       _dp]
        L.orc_fbk_euler_integrate.restype = ctypes.c_int
        L.orc_fbk_euler_integrate.argtypes = [ctypes.c_int, ctypes.c_double, _dp, _dp, _dp, _dp,
                                              _dp, ctypes.c_double, ctypes.c_double,
                                              ctypes.c_double]
        L.orc_fbd_euler_impedance_batch.restype = ctypes.c_int
        L.orc_fbd_euler_impedance_batch.argtypes = [
            ctypes.POINTER(OrcFbModel), ctypes.c_int64, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp,
            ctypes.c_int, _dp, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int]
        L.orc_fbd_com_batch.argtypes = [ctypes.POINTER(OrcFbModel), ctypes.c_int64, _dp, _dp, _dp,
                                        _dp, _dp, _dp]
        _LIB = L
    return _LIB


def _d(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def _i(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_ip)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def lti_euler_integrate(A, B, u, x, t0, t1, dT):
    A, B, u = _f64(A), _f64(B), _f64(u)
    x = _f64(x).copy()
    n, m = A.shape[0], B.shape[1]
    steps = ctypes.c_int64(0)
    st = lib().orc_lti_euler_integrate(n, m, _d(A), _d(B), _d(u), _d(x), t0, t1, dT,
                                       ctypes.byref(steps))
    return st, x, steps.value


def dcm_euler_rollout(xi0, omega, vrp, dt):
    xi0, omega, vrp = _f64(xi0), _f64(omega), _f64(vrp)
    N = omega.shape[0]
    out = np.zeros((N + 1, 2))
    lib().orc_dcm_euler_rollout(_d(xi0), _d(omega), _d(vrp), N, dt, _d(out))
    return out


def contact_phases(lists, max_phases=256):
    """lists: sequence of [(activation, deactivation), ...] per contact list (ordered)."""
    L = len(lists)
    C = max(1, max(len(l) for l in lists))
    act = np.zeros((L, C))
    deact = np.zeros((L, C))
    nc = np.zeros(L, dtype=np.int32)
    for l, lst in enumerate(lists):
        nc[l] = len(lst)
        for c, (a, d) in enumerate(lst):
            act[l, c], deact[l, c] = a, d
    begin = np.zeros(max_phases)
    end = np.zeros(max_phases)
    active = np.zeros((max_phases, L), dtype=np.int32)
    n = lib().orc_contact_phases(L, C, _d(act), _d(deact), _i(nc), max_phases, _d(begin),
                                 _d(end), _i(active))
    if n < 0:
        raise RuntimeError("too many phases")
    return begin[:n].copy(), end[:n].copy(), active[:n].copy()


def present_index(times, t):
    times = _f64(times)
    return lib().orc_present_index(_d(times), times.shape[0], t)


def hull2d_hrep(pts, max_facets=8):
    pts = _f64(pts)
    A = np.zeros((max_facets, 2))
    b = np.zeros(max_facets)
    m = lib().orc_hull2d_hrep(_d(pts), pts.shape[0], max_facets, _d(A), _d(b))
    return A, b, m


def hull2d_force_andrew(on):
    """Test switch: Andrew's monotone chain for every point count (orc_hull2d_force_andrew)."""
    lib().orc_hull2d_force_andrew(int(bool(on)))


def hull2d_contains(A, b, m, p):
    return bool(lib().orc_hull2d_contains(_d(_f64(A)), _d(_f64(b)), m, _d(_f64(p))))


def hull3d_hrep(pts, max_facets=64):
    """orc_hull3d_hrep: pts [p, 3] -> (A [max_facets, 3], b [max_facets], nfacets or -1)."""
    pts = _f64(pts)
    A = np.zeros((max_facets, 3))
    b = np.zeros(max_facets)
    m = lib().orc_hull3d_hrep(_d(pts), pts.shape[0], max_facets, _d(A), _d(b))
    return A, b, m


def hullnd_hrep(pts, max_facets=64):
    """orc_hullnd_hrep: pts [p, dim] -> (A [max_facets, dim], b [max_facets], nfacets or -1)."""
    pts = _f64(pts)
    p, dim = pts.shape
    A = np.zeros((max_facets, dim))
    b = np.zeros(max_facets)
    m = lib().orc_hullnd_hrep(dim, _d(pts), p, max_facets, _d(A), _d(b))
    return A, b, m


def halfspace_contains(A, b, m, p):
    A = _f64(A)
    return bool(lib().orc_halfspace_contains(_d(A), _d(_f64(b)), m, A.shape[-1], _d(_f64(p))))


def quintic_fit(knots_t, knots_pva):
    knots_t, knots_pva = _f64(knots_t), _f64(knots_pva)
    K1, dim = knots_t.shape[0], knots_pva.shape[2]
    coeffs = np.zeros((K1 - 1, dim, 6))
    lib().orc_quintic_fit(_d(knots_t), _d(knots_pva), K1, dim, _d(coeffs))
    return coeffs


def quintic_eval(knots_t, coeffs, tq):
    knots_t, coeffs, tq = _f64(knots_t), _f64(coeffs), _f64(tq)
    K1, dim = knots_t.shape[0], coeffs.shape[1]
    pva = np.zeros((tq.shape[0], 3, dim))
    idx = np.zeros(tq.shape[0], dtype=np.int32)
    lib().orc_quintic_eval(_d(knots_t), _d(coeffs), K1, dim, _d(tq), tq.shape[0], _d(pva),
                           _i(idx))
    return pva, idx


def default_params(horizon, **kw):
    p = OrcParams()
    p.horizon = horizon
    p.max_facets = kw.get("max_facets", 8)
    p.max_iter = kw.get("max_iter", 50)
    p.sequential = int(kw.get("sequential", 0))
    p.dt = kw.get("dt", 0.02)
    for name, val in (("w_xi", 1e2), ("w_vrp", 1.0), ("w_terminal", 1e3)):
        v = kw.get(name, val)
        getattr(p, name)[0] = v if np.isscalar(v) else v[0]
        getattr(p, name)[1] = v if np.isscalar(v) else v[1]
    p.tol_mu = kw.get("tol_mu", 1e-16)
    p.tol_primal = kw.get("tol_primal", 1e-10)
    p.tol_dual = kw.get("tol_dual", 1e-9)
    p.tol_polish = kw.get("tol_polish", 3e-4)   # blf_dcm_mpc_default_params
    # 1: evaluate as the device's BLF_QP_SINGLE_KERNEL=1 path (the IPM kernel alone)
    p.single_kernel = int(kw.get("single_kernel", 0))
    return p


# The device evaluates batches of at most this many QPs in its DPP scan tree (include/blf/blf_c.h
# BLF_DPP_TREE_MAX_BATCH); the oracle follows the same rule through orc_dcm_params.as_tree.
DPP_TREE_MAX_BATCH = 1024


def _tree_params(params, N, device_batch):
    """A copy of `params` (default_params(N) if None) with as_tree set for a device launch of
    `device_batch` QPs."""
    p = OrcParams()
    ctypes.memmove(ctypes.byref(p), ctypes.byref(params or default_params(N)), ctypes.sizeof(OrcParams))
    p.as_tree = 1 if device_batch <= DPP_TREE_MAX_BATCH else 0
    return p


def dcm_mpc_solve(prob, params=None, index=0, device_batch=None):
    """Solve problem `index` of a batch dict (keys as produced by blf.problems), as a device launch
    of `device_batch` QPs evaluates it (default: the dict's batch size)."""
    N = prob["omega"].shape[1]
    p = _tree_params(params, N, prob["omega"].shape[0] if device_batch is None else device_batch)
    xi = np.zeros((N + 1, 2))
    vrp = np.zeros((N, 2))
    it = np.zeros(1, dtype=np.int32)
    g = lambda k: np.ascontiguousarray(prob[k][index])
    st = lib().orc_dcm_mpc_solve(ctypes.byref(p), _d(g("xi_init")), _d(g("omega")),
                                 _d(g("xi_ref")), _d(g("vrp_ref")), _d(g("A")), _d(g("b")),
                                 _i(g("nfacets")), _d(xi), _d(vrp), _i(it))
    return st, xi, vrp, int(it[0])


def dcm_mpc_solve_batch(prob, params=None, threads=1, count=None, device_batch=None):
    """The first `count` problems (default: all), as a device launch of `device_batch` QPs
    evaluates them (default: the dict's batch size)."""
    B = prob["omega"].shape[0] if count is None else count
    N = prob["omega"].shape[1]
    p = _tree_params(params, N, prob["omega"].shape[0] if device_batch is None else device_batch)
    xi = np.zeros((B, N + 1, 2))
    vrp = np.zeros((B, N, 2))
    status = np.zeros(B, dtype=np.int32)
    iters = np.zeros(B, dtype=np.int32)
    g = lambda k: np.ascontiguousarray(prob[k][:B])
    lib().orc_dcm_mpc_solve_batch(ctypes.byref(p), B, threads, _d(g("xi_init")), _d(g("omega")),
                                  _d(g("xi_ref")), _d(g("vrp_ref")), _d(g("A")), _d(g("b")),
                                  _i(g("nfacets")), _d(xi), _d(vrp), _i(status), _i(iters))
    return status, xi, vrp, iters


def dcm_mpc_solve_batch_warm(prob, vrp_ws=None, lam_ws=None, shift=1, floor=1e-4,
                             params=None, threads=1, polished=None, prev_status=None, device_batch=None,
                             passes=None):
    """Batch solve from warm starts (vrp_ws [B][N][2], lam_ws [B][N][M]; None: cold starts;
    prev_status [B]: problems with a nonzero previous status start cold).
    Returns status, xi, vrp, iters, lam [B][N][M] (final multipliers); `polished` (an int32 [B]
    array, optional) receives whether the active-set polish was accepted, `passes` (int32 [B],
    optional) the active-set kernels' drop/add passes (blf_dcm_mpc_solution.passes)."""
    B, N = prob["omega"].shape
    p = _tree_params(params, N, B if device_batch is None else device_batch)
    M = p.max_facets
    xi = np.zeros((B, N + 1, 2))
    vrp = np.zeros((B, N, 2))
    lam = np.zeros((B, N, M))
    status = np.zeros(B, dtype=np.int32)
    iters = np.zeros(B, dtype=np.int32)
    g = lambda k: np.ascontiguousarray(prob[k])
    ws_v = None if vrp_ws is None else _f64(vrp_ws)
    ws_l = None if lam_ws is None else _f64(lam_ws)
    lib().orc_dcm_mpc_solve_batch_warm(
        ctypes.byref(p), B, threads, _d(g("xi_init")), _d(g("omega")), _d(g("xi_ref")),
        _d(g("vrp_ref")), _d(g("A")), _d(g("b")), _i(g("nfacets")),
        None if ws_v is None else _d(ws_v), None if ws_l is None else _d(ws_l),
        None if prev_status is None else _i(np.ascontiguousarray(prev_status, dtype=np.int32)), int(shift),
        float(floor), _d(xi), _d(vrp), _d(lam), _i(status), _i(iters),
        None if polished is None else _i(polished), None if passes is None else _i(passes))
    return status, xi, vrp, iters, lam


def dcm_phase_expand(table, start, dt, horizon):
    """table: nphases [B], phase_begin/phase_end [B,P], phase_A [B,P,M,2], phase_b [B,P,M],
    phase_nf [B,P], phase_ref [B,P,2] -> dict(A, b, nfacets, xi_ref, vrp_ref) of the window."""
    B, P = table["phase_begin"].shape
    M = table["phase_b"].shape[2]
    N = horizon
    out = dict(A=np.zeros((B, N, M, 2)), b=np.zeros((B, N, M)),
               nfacets=np.zeros((B, N), dtype=np.int32), xi_ref=np.zeros((B, N + 1, 2)),
               vrp_ref=np.zeros((B, N, 2)))
    c = lambda k, q: np.ascontiguousarray(table[k][q])
    for q in range(B):
        lib().orc_dcm_phase_expand(
            P, M, int(table["nphases"][q]), _d(c("phase_begin", q)), _d(c("phase_end", q)),
            _d(c("phase_A", q)), _d(c("phase_b", q)), _i(c("phase_nf", q)), _d(c("phase_ref", q)),
            int(start), float(dt), N, _d(out["A"][q]), _d(out["b"][q]), _i(out["nfacets"][q]),
            _d(out["xi_ref"][q]), _d(out["vrp_ref"][q]))
    return out


def hull2d_hrep_batch(pts, npts, max_facets=8, threads=1):
    """orc_hull2d_hrep over pts [count, P, 2] (npts [count] valid points each), threaded."""
    pts, npts = _f64(pts), np.ascontiguousarray(npts, dtype=np.int32)
    n, P = pts.shape[0], pts.shape[1]
    A = np.zeros((n, max_facets, 2))
    b = np.zeros((n, max_facets))
    nf = np.zeros(n, dtype=np.int32)
    lib().orc_hull2d_hrep_batch(n, P, max_facets, _d(pts), _i(npts), _d(A), _d(b), _i(nf), int(threads))
    return A, b, nf


def dcm_phase_expand_batch(table, start, dt, horizon, threads=1):
    """dcm_phase_expand with the C batch driver (threaded)."""
    B, P = table["phase_begin"].shape
    M = table["phase_b"].shape[2]
    N = horizon
    out = dict(A=np.zeros((B, N, M, 2)), b=np.zeros((B, N, M)),
               nfacets=np.zeros((B, N), dtype=np.int32), xi_ref=np.zeros((B, N + 1, 2)),
               vrp_ref=np.zeros((B, N, 2)))
    c = lambda k, dt_=np.float64: np.ascontiguousarray(table[k], dtype=dt_)
    lib().orc_dcm_phase_expand_batch(
        B, P, M, _i(c("nphases", np.int32)), _d(c("phase_begin")), _d(c("phase_end")),
        _d(c("phase_A")), _d(c("phase_b")), _i(c("phase_nf", np.int32)), _d(c("phase_ref")),
        int(start), float(dt), N, _d(out["A"]), _d(out["b"]), _i(out["nfacets"]), _d(out["xi_ref"]),
        _d(out["vrp_ref"]), int(threads))
    return out


def quintic_batch(knots_t, knots_pva, tq, threads=1):
    """Fit and evaluate S quintic splines (knots_t [S, K1], knots_pva [S, K1, 3, D], tq [S, Q])."""
    knots_t, knots_pva, tq = _f64(knots_t), _f64(knots_pva), _f64(tq)
    S, K1 = knots_t.shape
    D, Q = knots_pva.shape[3], tq.shape[1]
    coeffs = np.zeros((S, K1 - 1, D, 6))
    pva = np.zeros((S, Q, 3, D))
    idx = np.zeros((S, Q), dtype=np.int32)
    lib().orc_quintic_batch(S, K1, D, Q, _d(knots_t), _d(knots_pva), _d(tq), _d(coeffs), _d(pva),
                            _i(idx), int(threads))
    return coeffs, pva, idx


def wave_tree_sum(c):
    c = _f64(c)
    return lib().orc_wave_tree_sum(_d(c), c.shape[0])


def assemble_constraints(prob, max_facets=8):
    """Per-knot support polygon H-rep from the generator's corner sets, via the oracle hull."""
    corners, ncorners = prob["corners"], prob["ncorners"]
    B, N1 = ncorners.shape
    N = N1 - 1
    A = np.zeros((B, N, max_facets, 2))
    b = np.zeros((B, N, max_facets))
    m = np.zeros((B, N), dtype=np.int32)
    for i in range(B):
        for k in range(N):
            A[i, k], b[i, k], m[i, k] = hull2d_hrep(corners[i, k, :ncorners[i, k]], max_facets)
    out = dict(prob)
    out.update(A=A, b=b, nfacets=m)
    return out


# ---- config 5: ContinuousContactModel and FloatingBaseSystemKinematics ----------------------
def contact_eval(prm, twist, pose, null_pose):
    """One contact: returns wrench[6], autonomous[6], control[6,6], regressor[6,2]."""
    prm, twist, pose, null_pose = _f64(prm), _f64(twist), _f64(pose), _f64(null_pose)
    w, a, c, r = np.zeros(6), np.zeros(6), np.zeros(36), np.zeros(12)
    lib().orc_contact_eval(_d(prm), _d(twist), _d(pose), _d(null_pose), _d(w), _d(a), _d(c),
                           _d(r))
    return w, a, c.reshape(6, 6), r.reshape(6, 2)


def contact_eval_batch(prm, twist, pose, null_pose):
    """Batched: prm [B,4] (or [4]), twist [B,6], pose / null_pose [B,12]."""
    B = twist.shape[0]
    prm = np.broadcast_to(_f64(prm), (B, 4))
    out = [np.zeros((B, 6)), np.zeros((B, 6)), np.zeros((B, 6, 6)), np.zeros((B, 6, 2))]
    for q in range(B):
        res = contact_eval(prm[q], twist[q], pose[q], null_pose[q])
        for o, r in zip(out, res):
            o[q] = r
    return out


def contact_point(prm, twist, pose, null_pose, x, y):
    prm, twist, pose, null_pose = _f64(prm), _f64(twist), _f64(pose), _f64(null_pose)
    f, t = np.zeros(3), np.zeros(3)
    lib().orc_contact_point(_d(prm), _d(twist), _d(pose), _d(null_pose), float(x), float(y),
                            _d(f), _d(t))
    return f, t


def fbk_dynamics(rho, rot, twist, joint_vel):
    rot, twist, joint_vel = _f64(rot), _f64(twist), _f64(joint_vel)
    n = joint_vel.shape[0]
    dp, dR, dq = np.zeros(3), np.zeros(9), np.zeros(max(n, 1))
    lib().orc_fbk_dynamics(n, rho, _d(rot.reshape(-1)), _d(twist), _d(joint_vel if n else np.zeros(1)),
                           _d(dp), _d(dR), _d(dq))
    return dp, dR.reshape(3, 3), dq[:n]


def fbk_euler_integrate(rho, pos, rot, joints, twist, joint_vel, t0, t1, dT):
    pos, rot, joints = _f64(pos).copy(), _f64(rot).reshape(-1).copy(), _f64(joints).copy()
    twist, joint_vel = _f64(twist), _f64(joint_vel)
    n = joints.shape[0]
    jz = joints if n else np.zeros(1)
    jv = joint_vel if n else np.zeros(1)
    st = lib().orc_fbk_euler_integrate(n, rho, _d(pos), _d(rot), _d(jz), _d(twist), _d(jv),
                                       t0, t1, dT)
    return st, pos, rot.reshape(3, 3), joints


def fbd_euler_impedance_batch(model, states, q_ref, kp, kd, contact_params, null_poses, t0, t1, dT,
                              rho=0.01, gravity=(0.0, 0.0, -9.81), threads=1):
    """C restatement (blf_oracle_fbd.c) of fb_dynamics / closed_loop.euler_integrate_impedance for
    B robots: states dict of [B,...] arrays (base_pos, base_rot [B,3,3], joint_pos, base_vel,
    joint_vel), q_ref [B,n], kp / kd [n], contact_params [C,4], null_poses [B,C,12].  Returns the
    integrated states (new arrays)."""
    keep = []

    def arr(a, dt=np.float64):
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a
    mdl = _fb_model(model, keep, rho, gravity)
    out = {k: np.array(states[k], dtype=np.float64, copy=True)
           for k in ("base_pos", "base_rot", "joint_pos", "base_vel", "joint_vel")}
    B = out["base_pos"].shape[0]
    cp, npz = arr(contact_params), arr(null_poses)
    rc = lib().orc_fbd_euler_impedance_batch(
        ctypes.byref(mdl), B, _d(out["base_pos"]), _d(out["base_rot"]), _d(out["joint_pos"]),
        _d(out["base_vel"]), _d(out["joint_vel"]), _d(arr(q_ref)), _d(arr(kp)), _d(arr(kd)),
        int(cp.shape[0]), _d(cp), _d(npz), t0, t1, dT, threads)
    if rc:
        raise RuntimeError(f"orc_fbd_euler_impedance_batch failed ({rc})")
    return out


def _fb_model(model, keep, rho=0.01, gravity=(0.0, 0.0, -9.81)):
    def arr(a, dt=np.float64):
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a
    return OrcFbModel(int(model["n"]), _i(arr(model["parent"], np.int32)),
                      _d(arr(model["joint_origin"])), _d(arr(model["joint_rot"])),
                      _d(arr(model["joint_axis"])), _d(arr(model["link_mass"])),
                      _d(arr(model["link_com"])), _d(arr(model["link_inertia"])),
                      _i(arr(model["frame_link"], np.int32)), _d(arr(model["frame_pose"])),
                      (ctypes.c_double * 3)(*gravity), rho,
                      None if model.get("joint_type") is None else _i(arr(model["joint_type"], np.int32)))


def fbd_com_batch(model, states):
    """C restatement of closed_loop.com_state for B robots: com [B,6] = (c, cdot)."""
    keep = []
    mdl = _fb_model(model, keep)
    st = {k: np.ascontiguousarray(states[k], dtype=np.float64)
          for k in ("base_pos", "base_rot", "joint_pos", "base_vel", "joint_vel")}
    B = st["base_pos"].shape[0]
    com = np.zeros((B, 6))
    lib().orc_fbd_com_batch(ctypes.byref(mdl), B, _d(st["base_pos"]), _d(st["base_rot"]),
                            _d(st["joint_pos"]), _d(st["base_vel"]), _d(st["joint_vel"]), _d(com))
    return com
