"""ctypes binding of the C ABI in include/blf/blf_c.h (lib/libblf.so, built for gfx950).

torch is used only as device-memory and stream plumbing: every function takes torch CUDA
tensors, checks dtype/shape/contiguity/device on the host, and passes raw device pointers plus
torch's current HIP stream to the library.  There is no CPU fallback: if lib/libblf.so is
missing or cannot be loaded, `lib()` raises, and every op raises with it.
"""
import ctypes
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG, "lib", "libblf.so")
# diagnostic builds only (tools/kbench.py): BLF_LIB points at e.g. lib/libblf_stamps.so
LIB_PATH = os.environ.get("BLF_LIB", LIB_PATH)

BLF_OK = 0
STATUS_NAMES = {0: "BLF_OK", 1: "BLF_ERR_INVALID_ARGUMENT", 2: "BLF_ERR_HIP",
                3: "BLF_ERR_UNSUPPORTED", 4: "BLF_ERR_TIME_INTERVAL", 5: "BLF_ERR_EMPTY_INTERVAL"}
QP_SOLVED, QP_MAX_ITER, QP_NUMERICAL, QP_BAD_FACETS = 0, 1, 2, 3

# every symbol include/blf/blf_c.h declares (tests/test_abi.py checks the .so exports them)
EXPORTED = ["blf_create", "blf_destroy", "blf_last_error", "blf_version", "blf_set_qp_launch_mode",
            "blf_step_schedule",
            "blf_lti_euler_integrate", "blf_lti_dynamics", "blf_dcm_euler_rollout", "blf_hull2d_hrep",
            "blf_hull2d_contains", "blf_hull3d_hrep", "blf_hullnd_hrep", "blf_halfspace_contains", "blf_quintic_fit", "blf_quintic_eval",
            "blf_dcm_mpc_default_params", "blf_dcm_mpc_solve", "blf_dcm_mpc_solve_warm",
            "blf_dcm_phase_expand", "blf_dcm_mpc_solve_phased",
            "blf_dcm_mpc_flops_per_iter",
            "blf_contact_model_eval", "blf_contact_point_wrench", "blf_fbk_dynamics",
            "blf_fbk_euler_integrate", "blf_fbd_dynamics", "blf_fbd_euler_integrate",
            "blf_fb_dcm", "blf_dcm_posture_reference", "blf_fbd_euler_integrate_impedance",
            "blf_fb_frame_state"]
# entry points removed in round 5 (measured slower, never the default; tests/test_abi.py checks
# that the library no longer exports them)
REMOVED = ["blf_set_qp_split_batch", "blf_stream_create_cu_range", "blf_stream_destroy",
           "blf_dcm_mpc_solve_phased_begin", "blf_dcm_mpc_solve_phased_finish",
           "blf_dcm_posture_reference_masked", "blf_fbd_euler_integrate_impedance_masked"]

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f64 = ctypes.c_double


class FbModel(ctypes.Structure):
    """blf_fb_model (include/blf/blf_c.h); every pointer is device memory."""
    _fields_ = [("ndof", _i32), ("nframes", _i32), ("parent", _vp), ("joint_origin", _vp),
                ("joint_rot", _vp), ("joint_axis", _vp), ("link_mass", _vp), ("link_com", _vp),
                ("link_inertia", _vp), ("frame_link", _vp), ("frame_pose", _vp),
                ("gravity", _f64 * 3), ("rho", _f64), ("joint_type", _vp)]


class FbState(ctypes.Structure):
    _fields_ = [("base_vel", _vp), ("joint_vel", _vp), ("base_pos", _vp), ("base_rot", _vp),
                ("joint_pos", _vp)]


CONTACT_CONTINUOUS, CONTACT_WRENCH = 0, 1   # blf_fb_contacts.law (BLF_CONTACT_*)


class FbContacts(ctypes.Structure):
    _fields_ = [("ncontacts", _i32), ("frame", _vp), ("params", _vp), ("null_pose", _vp),
                ("law", _vp), ("wrench", _vp)]


class PostureLaw(ctypes.Structure):
    """blf_posture_law (include/blf/blf_c.h): the closed loop's plan -> joint reference map."""
    _fields_ = [("ndof", _i32), ("reserved", _i32), ("q_nominal", _vp), ("lean", _vp)]


class JointImpedance(ctypes.Structure):
    """blf_joint_impedance: tau = kp (q_ref - q) - kd qdot before every Euler step."""
    _fields_ = [("ndof", _i32), ("reserved", _i32), ("kp", _vp), ("kd", _vp), ("q_ref", _vp)]


FB_STATE_KEYS = ("base_vel", "joint_vel", "base_pos", "base_rot", "joint_pos")


class BlfError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


class DcmMpcParams(ctypes.Structure):
    _fields_ = [("horizon", _i32), ("max_facets", _i32), ("max_iter", _i32), ("reserved", _i32),
                ("dt", _f64), ("w_xi", _f64 * 2), ("w_vrp", _f64 * 2), ("w_terminal", _f64 * 2),
                ("tol_mu", _f64), ("tol_primal", _f64), ("tol_dual", _f64), ("tol_polish", _f64)]


class DcmMpcProblem(ctypes.Structure):
    _fields_ = [("xi_init", _vp), ("omega", _vp), ("xi_ref", _vp), ("vrp_ref", _vp), ("A", _vp),
                ("b", _vp), ("nfacets", _vp)]


class DcmMpcSolution(ctypes.Structure):
    _fields_ = [("xi", _vp), ("vrp", _vp), ("status", _vp), ("iters", _vp), ("polished", _vp),
                ("passes", _vp)]


class PhaseTable(ctypes.Structure):
    _fields_ = [("max_phases", _i32), ("max_facets", _i32), ("nphases", _vp), ("begin", _vp),
                ("end", _vp), ("A", _vp), ("b", _vp), ("nfacets", _vp), ("ref", _vp)]


class DcmMpcWindow(ctypes.Structure):
    _fields_ = [("omega", _vp), ("xi_ref", _vp), ("vrp_ref", _vp), ("A", _vp), ("b", _vp),
                ("nfacets", _vp)]


class DcmMpcWarmStart(ctypes.Structure):
    _fields_ = [("vrp", _vp), ("lambda_", _vp), ("shift", _i32), ("reserved", _i32),
                ("floor", _f64), ("prev_status", _vp)]


def _warm_start(warm, B, N, M):
    """blf_dcm_mpc_warm_start from a dict: vrp [B,N,2], lam [B,N,M], shift, floor and optionally
    status [B] int32 (the previous solve's statuses: problems with status != 0 start cold)."""
    torch = _torch()
    st = warm.get("status")
    return DcmMpcWarmStart(_ptr(warm["vrp"], torch.float64, (B, N, 2), "warm vrp"),
                           _ptr(warm["lam"], torch.float64, (B, N, M), "warm lam"),
                           int(warm.get("shift", 1)), 0, float(warm.get("floor", 1e-2)),
                           _ptr(st, torch.int32, (B,), "warm status") if st is not None else None)


_LIB = None


def lib():
    """Load lib/libblf.so (raises if it is absent: there is no fallback path)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C "
                              f"bipedal-locomotion-framework_amd)")
        # One HIP runtime per process: libblf.so needs libamdhip64.so.7, and torch ships its own
        # copy.  Loaded after torch, libblf.so binds to torch's (same soname) and shares its
        # device memory and streams; loaded first, the process would hold two runtimes and the
        # one that initialises second sees no device.  So torch, when installed, is loaded first.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.blf_create.argtypes = [ctypes.POINTER(_vp), _i32]
        L.blf_destroy.argtypes = [_vp]
        L.blf_last_error.restype = ctypes.c_char_p
        L.blf_version.restype = ctypes.c_char_p
        L.blf_lti_euler_integrate.argtypes = [_vp, _i32, _i32, _vp, _vp, _i32, _vp, _vp, _i64,
                                              _f64, _f64, _f64, _vp]
        L.blf_lti_dynamics.argtypes = [_vp, _i32, _i32, _vp, _vp, _i32, _vp, _vp, _vp, _i64, _vp]
        L.blf_dcm_euler_rollout.argtypes = [_vp, _vp, _vp, _vp, _i32, _f64, _vp, _i64, _vp]
        L.blf_hull2d_hrep.argtypes = [_vp, _vp, _vp, _i32, _i32, _i64, _vp, _vp, _vp, _vp]
        L.blf_hull2d_contains.argtypes = [_vp, _vp, _vp, _vp, _i32, _vp, _i64, _vp, _vp]
        L.blf_hull3d_hrep.argtypes = [_vp, _vp, _vp, _i32, _i32, _i64, _vp, _vp, _vp, _vp]
        L.blf_hullnd_hrep.argtypes = [_vp, _i32, _vp, _vp, _i32, _i32, _i64, _vp, _vp, _vp, _vp]
        L.blf_halfspace_contains.argtypes = [_vp, _vp, _vp, _vp, _i32, _i32, _vp, _i64, _vp, _vp]
        L.blf_quintic_fit.argtypes = [_vp, _vp, _vp, _i32, _i32, _i64, _vp, _vp]
        L.blf_quintic_eval.argtypes = [_vp, _vp, _vp, _i32, _i32, _i64, _vp, _i32, _vp, _vp, _vp]
        L.blf_dcm_mpc_default_params.argtypes = [ctypes.POINTER(DcmMpcParams), _i32]
        L.blf_dcm_mpc_default_params.restype = None
        L.blf_dcm_mpc_solve.argtypes = [_vp, ctypes.POINTER(DcmMpcParams),
                                        ctypes.POINTER(DcmMpcProblem), _i64,
                                        ctypes.POINTER(DcmMpcSolution), _vp]
        L.blf_dcm_mpc_solve_warm.argtypes = [_vp, ctypes.POINTER(DcmMpcParams),
                                             ctypes.POINTER(DcmMpcProblem),
                                             ctypes.POINTER(DcmMpcWarmStart), _i64,
                                             ctypes.POINTER(DcmMpcSolution), _vp, _vp]
        L.blf_dcm_phase_expand.argtypes = [_vp, ctypes.POINTER(PhaseTable), _i64, _f64, _i32,
                                           _i64, _vp, _vp, _vp, _vp, _vp, _vp]
        L.blf_dcm_mpc_solve_phased.argtypes = [_vp, ctypes.POINTER(DcmMpcParams),
                                               ctypes.POINTER(PhaseTable), _i64, _vp, _vp, _i64,
                                               ctypes.POINTER(DcmMpcWarmStart), _i64,
                                               ctypes.POINTER(DcmMpcWindow),
                                               ctypes.POINTER(DcmMpcSolution), _vp, _vp]
        L.blf_dcm_mpc_flops_per_iter.argtypes = [_i32, _i64]
        L.blf_contact_model_eval.argtypes = [_vp, _vp, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                             _vp, _vp]
        L.blf_contact_point_wrench.argtypes = [_vp, _vp, _i32, _vp, _vp, _vp, _i64, _vp, _i32,
                                               _vp, _vp, _vp]
        L.blf_fbk_dynamics.argtypes = [_vp, _i32, _f64, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]
        L.blf_fbk_euler_integrate.argtypes = [_vp, _i32, _f64, _vp, _vp, _vp, _vp, _vp, _i64,
                                              _f64, _f64, _f64, _vp]
        L.blf_fbd_dynamics.argtypes = [_vp, ctypes.POINTER(FbModel), ctypes.POINTER(FbState), _vp,
                                       ctypes.POINTER(FbContacts), _vp, _i64,
                                       ctypes.POINTER(FbState), _vp]
        L.blf_fbd_euler_integrate.argtypes = [_vp, ctypes.POINTER(FbModel), ctypes.POINTER(FbState),
                                              _vp, ctypes.POINTER(FbContacts), _vp, _i64, _f64,
                                              _f64, _f64, _vp]
        L.blf_fb_dcm.argtypes = [_vp, ctypes.POINTER(FbModel), ctypes.POINTER(FbState), _vp, _i64,
                                 _i64, _vp, _vp, _vp]
        L.blf_dcm_posture_reference.argtypes = [_vp, ctypes.POINTER(PostureLaw), _vp, _vp, _i64, _i64,
                                                _vp, _vp]
        L.blf_fbd_euler_integrate_impedance.argtypes = [
            _vp, ctypes.POINTER(FbModel), ctypes.POINTER(FbState), ctypes.POINTER(JointImpedance),
            ctypes.POINTER(FbContacts), _vp, _i64, _f64, _f64, _f64, _vp]
        L.blf_fb_frame_state.argtypes = [_vp, ctypes.POINTER(FbModel), ctypes.POINTER(FbState), _i32,
                                         _vp, _i64, _vp, _vp, _vp]
        L.blf_dcm_mpc_flops_per_iter.restype = _f64
        L.blf_set_qp_launch_mode.argtypes = [_i32, _i32]
        for name in EXPORTED:
            if name not in ("blf_create", "blf_destroy", "blf_last_error", "blf_version",
                            "blf_dcm_mpc_default_params", "blf_dcm_mpc_flops_per_iter"):
                getattr(L, name).restype = _i32
        L.blf_create.restype = _i32
        L.blf_destroy.restype = _i32
        _LIB = L
    return _LIB


def set_qp_launch_mode(fuse_stage2=-1, single_kernel=-1):
    """blf_set_qp_launch_mode: the QP kernel routing for A/B and parity tests (-1: unchanged).
    Returns nothing; the defaults are the product's (fuse_stage2 = 1, single_kernel = 0)."""
    _check(lib().blf_set_qp_launch_mode(int(fuse_stage2), int(single_kernel)))


def _check(code):
    if code != BLF_OK:
        raise BlfError(code, lib().blf_last_error().decode())


def last_error():
    return lib().blf_last_error().decode()


def version():
    return lib().blf_version().decode()


def source_hash():
    """The Makefile's SRC_HASH of the kernel / C-ABI sources in this tree (sha256 of csrc/*.hip and
    csrc/*.h in sorted path order, then include/blf/blf_c.h; first 16 hex digits), or None when
    the sources are not present."""
    import glob
    import hashlib
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    names = sorted(os.path.relpath(f, pkg) for f in glob.glob(os.path.join(pkg, "csrc", "*.hip")) +
                   glob.glob(os.path.join(pkg, "csrc", "*.h")))
    hdr = os.path.join(os.path.dirname(pkg), "include", "blf", "blf_c.h")
    if not names or not os.path.exists(hdr):
        return None
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(pkg, n), "rb") as f:
            h.update(f.read())
    with open(hdr, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def build_provenance():
    """Which library this process loaded and whether it was built from the sources in this tree:
    {"lib": path, "lib_src_hash": hash in blf_version(), "tree_src_hash": source_hash(),
    "matches": bool}."""
    v = version()
    lib_hash = v.rsplit(" src ", 1)[1] if " src " in v else None
    tree = source_hash()
    return {"lib": LIB_PATH, "lib_src_hash": lib_hash, "tree_src_hash": tree,
            "matches": lib_hash is not None and lib_hash == tree}


def default_params(horizon, **kw):
    p = DcmMpcParams()
    lib().blf_dcm_mpc_default_params(ctypes.byref(p), horizon)
    for k, v in kw.items():
        if k in ("w_xi", "w_vrp", "w_terminal"):
            arr = getattr(p, k)
            arr[0], arr[1] = (v, v) if isinstance(v, (int, float)) else (v[0], v[1])
        else:
            setattr(p, k, v)
    return p


def flops_per_iter(horizon, active_facets):
    return lib().blf_dcm_mpc_flops_per_iter(horizon, active_facets)


# ---------------------------------------------------------------------------------------------
# device-side helpers (torch as plumbing)
# ---------------------------------------------------------------------------------------------
def _torch():
    import torch
    return torch


def _ptr(t, dtype, shape=None, name="tensor"):
    torch = _torch()
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a device (cuda/hip) tensor, got {t.device}")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    return _vp(t.data_ptr())


def _stream(stream=None):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return _vp(s.cuda_stream)


class Handle:
    """RAII wrapper of blf_handle (one per device per thread)."""

    def __init__(self, device=0):
        self._h = _vp()
        _check(lib().blf_create(ctypes.byref(self._h), device))
        self.device = device

    def close(self):
        if self._h:
            lib().blf_destroy(self._h)
            self._h = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ptr(self):
        return self._h

    # --- ForwardEuler<LinearTimeInvariantSystem>::integrate, batched, in place on x ---
    def lti_euler_integrate(self, A, Bm, u, x, t0, t1, dT, shared=False, stream=None):
        torch = _torch()
        n = x.shape[-1]
        m = u.shape[-1]
        batch = x.shape[0]
        ashape = (n, n) if shared else (batch, n, n)
        bshape = (n, m) if shared else (batch, n, m)
        _check(lib().blf_lti_euler_integrate(
            self._h, n, m, _ptr(A, torch.float64, ashape, "A"), _ptr(Bm, torch.float64, bshape, "B"),
            1 if shared else 0, _ptr(u, torch.float64, (batch, m), "u"),
            _ptr(x, torch.float64, (batch, n), "x"), batch, t0, t1, dT, _stream(stream)))
        return x

    def lti_dynamics(self, A, Bm, u, x, shared=False, stream=None):
        torch = _torch()
        batch, n = x.shape
        m = u.shape[-1]
        ashape = (n, n) if shared else (batch, n, n)
        bshape = (n, m) if shared else (batch, n, m)
        dx = torch.empty_like(x)
        _check(lib().blf_lti_dynamics(
            self._h, n, m, _ptr(A, torch.float64, ashape, "A"), _ptr(Bm, torch.float64, bshape, "B"),
            1 if shared else 0, _ptr(u, torch.float64, (batch, m), "u"),
            _ptr(x, torch.float64, (batch, n), "x"), _ptr(dx, torch.float64, (batch, n), "dx"),
            batch, _stream(stream)))
        return dx

    def dcm_euler_rollout(self, xi0, omega, vrp, dt, out=None, stream=None):
        torch = _torch()
        B, N = omega.shape
        if out is None:
            out = torch.empty((B, N + 1, 2), dtype=torch.float64, device=omega.device)
        _check(lib().blf_dcm_euler_rollout(
            self._h, _ptr(xi0, torch.float64, (B, 2), "xi0"), _ptr(omega, torch.float64, (B, N), "omega"),
            _ptr(vrp, torch.float64, (B, N, 2), "vrp"), N, dt,
            _ptr(out, torch.float64, (B, N + 1, 2), "xi_out"), B, _stream(stream)))
        return out

    def hull2d_hrep(self, pts, npts, max_facets=8, out=None, stream=None):
        torch = _torch()
        B, P = pts.shape[0], pts.shape[1]
        if out is None:
            out = (torch.empty((B, max_facets, 2), dtype=torch.float64, device=pts.device),
                   torch.empty((B, max_facets), dtype=torch.float64, device=pts.device),
                   torch.empty((B,), dtype=torch.int32, device=pts.device))
        A, b, nf = out
        _check(lib().blf_hull2d_hrep(
            self._h, _ptr(pts, torch.float64, (B, P, 2), "pts"), _ptr(npts, torch.int32, (B,), "npts"),
            P, max_facets, B, _ptr(A, torch.float64, (B, max_facets, 2), "A"),
            _ptr(b, torch.float64, (B, max_facets), "b"), _ptr(nf, torch.int32, (B,), "nfacets"),
            _stream(stream)))
        return A, b, nf

    def hullnd_hrep(self, pts, npts, max_facets=64, out=None, stream=None):
        """blf_hullnd_hrep: pts [B, P, dim], npts [B] -> A [B, max_facets, dim], b, nfacets."""
        torch = _torch()
        B, P, D = pts.shape
        if out is None:
            out = (torch.empty((B, max_facets, D), dtype=torch.float64, device=pts.device),
                   torch.empty((B, max_facets), dtype=torch.float64, device=pts.device),
                   torch.empty((B,), dtype=torch.int32, device=pts.device))
        A, b, nf = out
        _check(lib().blf_hullnd_hrep(
            self._h, D, _ptr(pts, torch.float64, (B, P, D), "pts"), _ptr(npts, torch.int32, (B,), "npts"),
            P, max_facets, B, _ptr(A, torch.float64, (B, max_facets, D), "A"),
            _ptr(b, torch.float64, (B, max_facets), "b"), _ptr(nf, torch.int32, (B,), "nfacets"),
            _stream(stream)))
        return A, b, nf

    def hull2d_contains(self, A, b, nf, query, stream=None):
        torch = _torch()
        B, M = b.shape
        inside = torch.empty((B,), dtype=torch.int32, device=A.device)
        _check(lib().blf_hull2d_contains(
            self._h, _ptr(A, torch.float64, (B, M, 2), "A"), _ptr(b, torch.float64, (B, M), "b"),
            _ptr(nf, torch.int32, (B,), "nfacets"), M, _ptr(query, torch.float64, (B, 2), "query"),
            B, _ptr(inside, torch.int32, (B,), "inside"), _stream(stream)))
        return inside

    def hull3d_hrep(self, pts, npts, max_facets=32, out=None, stream=None):
        """blf_hull3d_hrep: pts [B, P, 3], npts [B] -> A [B, max_facets, 3], b, nfacets."""
        torch = _torch()
        B, P = pts.shape[0], pts.shape[1]
        if out is None:
            out = (torch.empty((B, max_facets, 3), dtype=torch.float64, device=pts.device),
                   torch.empty((B, max_facets), dtype=torch.float64, device=pts.device),
                   torch.empty((B,), dtype=torch.int32, device=pts.device))
        A, b, nf = out
        _check(lib().blf_hull3d_hrep(
            self._h, _ptr(pts, torch.float64, (B, P, 3), "pts"), _ptr(npts, torch.int32, (B,), "npts"),
            P, max_facets, B, _ptr(A, torch.float64, (B, max_facets, 3), "A"),
            _ptr(b, torch.float64, (B, max_facets), "b"), _ptr(nf, torch.int32, (B,), "nfacets"),
            _stream(stream)))
        return A, b, nf

    def halfspace_contains(self, A, b, nf, query, stream=None):
        """blf_halfspace_contains: A [B, M, dim], b [B, M], nf [B], query [B, dim] -> inside [B]."""
        torch = _torch()
        B, M, D = A.shape
        inside = torch.empty((B,), dtype=torch.int32, device=A.device)
        _check(lib().blf_halfspace_contains(
            self._h, _ptr(A, torch.float64, (B, M, D), "A"), _ptr(b, torch.float64, (B, M), "b"),
            _ptr(nf, torch.int32, (B,), "nfacets"), D, M, _ptr(query, torch.float64, (B, D), "query"),
            B, _ptr(inside, torch.int32, (B,), "inside"), _stream(stream)))
        return inside

    def quintic_fit(self, knots_t, knots_pva, stream=None):
        torch = _torch()
        S, K1 = knots_t.shape
        D = knots_pva.shape[-1]
        coeffs = torch.empty((S, K1 - 1, D, 6), dtype=torch.float64, device=knots_t.device)
        _check(lib().blf_quintic_fit(
            self._h, _ptr(knots_t, torch.float64, (S, K1), "knots_t"),
            _ptr(knots_pva, torch.float64, (S, K1, 3, D), "knots_pva"), K1, D, S,
            _ptr(coeffs, torch.float64, (S, K1 - 1, D, 6), "coeffs"), _stream(stream)))
        return coeffs

    def quintic_eval(self, knots_t, coeffs, tq, stream=None):
        torch = _torch()
        S, K1 = knots_t.shape
        D = coeffs.shape[2]
        Q = tq.shape[1]
        pva = torch.empty((S, Q, 3, D), dtype=torch.float64, device=tq.device)
        idx = torch.empty((S, Q), dtype=torch.int32, device=tq.device)
        _check(lib().blf_quintic_eval(
            self._h, _ptr(knots_t, torch.float64, (S, K1), "knots_t"),
            _ptr(coeffs, torch.float64, (S, K1 - 1, D, 6), "coeffs"), K1, D, S,
            _ptr(tq, torch.float64, (S, Q), "tq"), Q, _ptr(pva, torch.float64, (S, Q, 3, D), "pva"),
            _ptr(idx, torch.int32, (S, Q), "knot_idx"), _stream(stream)))
        return pva, idx

    def dcm_mpc_solve(self, prob, params=None, out=None, stream=None, warm=None,
                      lambda_out=False):
        """prob: dict of device tensors xi_init [B,2], omega [B,N], xi_ref [B,N+1,2],
        vrp_ref [B,N,2], A [B,N,M,2], b [B,N,M], nfacets [B,N] (int32).
        warm: None (cold start) or dict(vrp [B,N,2], lam [B,N,M], shift, floor)
        (blf_dcm_mpc_solve_warm); lambda_out: also return the final multipliers out["lam"].
        out["polished"] [B] says which solutions are the certified active-set polish; out["passes"]
        [B] how many drop/add passes the active-set kernels ran for each."""
        torch = _torch()
        B, N = prob["omega"].shape
        M = prob["b"].shape[2]
        p = params if params is not None else default_params(N, max_facets=M)
        if p.horizon != N or p.max_facets != M:
            raise ValueError("params.horizon / max_facets do not match the problem arrays")
        dev = prob["omega"].device
        if out is None:
            out = dict(xi=torch.empty((B, N + 1, 2), dtype=torch.float64, device=dev),
                       vrp=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
                       status=torch.empty((B,), dtype=torch.int32, device=dev),
                       iters=torch.empty((B,), dtype=torch.int32, device=dev),
                       polished=torch.empty((B,), dtype=torch.int32, device=dev),
                       passes=torch.empty((B,), dtype=torch.int32, device=dev))
        pb = DcmMpcProblem(
            _ptr(prob["xi_init"], torch.float64, (B, 2), "xi_init"),
            _ptr(prob["omega"], torch.float64, (B, N), "omega"),
            _ptr(prob["xi_ref"], torch.float64, (B, N + 1, 2), "xi_ref"),
            _ptr(prob["vrp_ref"], torch.float64, (B, N, 2), "vrp_ref"),
            _ptr(prob["A"], torch.float64, (B, N, M, 2), "A"),
            _ptr(prob["b"], torch.float64, (B, N, M), "b"),
            _ptr(prob["nfacets"], torch.int32, (B, N), "nfacets"))
        so = DcmMpcSolution(
            _ptr(out["xi"], torch.float64, (B, N + 1, 2), "xi"),
            _ptr(out["vrp"], torch.float64, (B, N, 2), "vrp"),
            _ptr(out["status"], torch.int32, (B,), "status"),
            _ptr(out["iters"], torch.int32, (B,), "iters"),
            _ptr(out["polished"], torch.int32, (B,), "polished") if "polished" in out else None,
            _ptr(out["passes"], torch.int32, (B,), "passes") if "passes" in out else None)
        ws = None
        if warm is not None:
            ws = _warm_start(warm, B, N, M)
        lam_ptr = None
        if lambda_out:
            if "lam" not in out:
                out["lam"] = torch.empty((B, N, M), dtype=torch.float64, device=dev)
            lam_ptr = _ptr(out["lam"], torch.float64, (B, N, M), "lam")
        self._keep = (pb, so, ws)
        if ws is None and lam_ptr is None:
            _check(lib().blf_dcm_mpc_solve(self._h, ctypes.byref(p), ctypes.byref(pb), B,
                                           ctypes.byref(so), _stream(stream)))
        else:
            _check(lib().blf_dcm_mpc_solve_warm(
                self._h, ctypes.byref(p), ctypes.byref(pb),
                ctypes.byref(ws) if ws is not None else None, B, ctypes.byref(so), lam_ptr,
                _stream(stream)))
        return out

    def prepare_dcm_mpc_solve(self, prob, params, out, stream=None):
        """The cold blf_dcm_mpc_solve with its argument structs built once: returns f(), which
        makes just the C-ABI call (what a C++ caller holding its device buffers pays, e.g. the
        TimeVaryingDCMPlanner adapter), and the raw stream handle.  The tensors must outlive f."""
        torch = _torch()
        self.dcm_mpc_solve(prob, params, out=out, stream=stream)   # validates every argument
        B, N = prob["omega"].shape
        M = prob["b"].shape[2]
        pb = DcmMpcProblem(*(_vp(prob[k].data_ptr()) for k in
                             ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")))
        so = DcmMpcSolution(*(_vp(out[k].data_ptr()) if k in out else None
                              for k in ("xi", "vrp", "status", "iters", "polished", "passes")))
        s = _stream(stream)
        fn, h, pp, ppb, pso = lib().blf_dcm_mpc_solve, self._h, ctypes.byref(params), ctypes.byref(pb), ctypes.byref(so)
        keep = (pb, so, params, prob, out, torch)

        def f():
            st = fn(h, pp, ppb, B, pso, s)
            if st != 0:
                _check(st)
            return keep
        return f, s

    def phase_table(self, nphases, begin, end, corners, ncorners, max_facets=8, ref=None,
                    stream=None):
        """Device phase table: the H-rep of every phase's support polygon (blf_hull2d_hrep over
        corners [B,P,C,2] / ncorners [B,P]) plus the phases' times and centroid references.
        ref [B,P,2]: the phases' reference points (default: the centroid of the corners)."""
        torch = _torch()
        B, P, C, _ = corners.shape
        A, b, nf = self.hull2d_hrep(corners.reshape(B * P, C, 2).contiguous(),
                                    ncorners.reshape(B * P).contiguous(), max_facets,
                                    stream=stream)
        if ref is None:
            cnt = ncorners.to(torch.float64).clamp(min=1)[..., None]
            ref = (corners.sum(dim=2) / cnt).contiguous()
        return dict(nphases=nphases, phase_begin=begin, phase_end=end,
                    phase_A=A.view(B, P, max_facets, 2), phase_b=b.view(B, P, max_facets),
                    phase_nf=nf.view(B, P), phase_ref=ref)

    def dcm_phase_expand(self, table, start, dt, horizon, out=None, stream=None):
        """blf_dcm_phase_expand: window arrays (A, b, nfacets, xi_ref, vrp_ref) of knots
        (start + k) dt, k = 0..horizon, from a phase table (phase_table() or the same keys)."""
        torch = _torch()
        B, P = table["phase_begin"].shape
        M = table["phase_b"].shape[2]
        N = horizon
        dev = table["phase_begin"].device
        if out is None:
            out = dict(A=torch.empty((B, N, M, 2), dtype=torch.float64, device=dev),
                       b=torch.empty((B, N, M), dtype=torch.float64, device=dev),
                       nfacets=torch.empty((B, N), dtype=torch.int32, device=dev),
                       xi_ref=torch.empty((B, N + 1, 2), dtype=torch.float64, device=dev),
                       vrp_ref=torch.empty((B, N, 2), dtype=torch.float64, device=dev))
        tb = PhaseTable(P, M, _ptr(table["nphases"], torch.int32, (B,), "nphases"),
                        _ptr(table["phase_begin"], torch.float64, (B, P), "phase_begin"),
                        _ptr(table["phase_end"], torch.float64, (B, P), "phase_end"),
                        _ptr(table["phase_A"], torch.float64, (B, P, M, 2), "phase_A"),
                        _ptr(table["phase_b"], torch.float64, (B, P, M), "phase_b"),
                        _ptr(table["phase_nf"], torch.int32, (B, P), "phase_nf"),
                        _ptr(table["phase_ref"], torch.float64, (B, P, 2), "phase_ref"))
        self._keep = tb
        _check(lib().blf_dcm_phase_expand(
            self._h, ctypes.byref(tb), int(start), float(dt), N, B,
            _ptr(out["A"], torch.float64, (B, N, M, 2), "A"),
            _ptr(out["b"], torch.float64, (B, N, M), "b"),
            _ptr(out["nfacets"], torch.int32, (B, N), "nfacets"),
            _ptr(out["xi_ref"], torch.float64, (B, N + 1, 2), "xi_ref"),
            _ptr(out["vrp_ref"], torch.float64, (B, N, 2), "vrp_ref"), _stream(stream)))
        return out

    def _phase_table_struct(self, table):
        torch = _torch()
        B, P = table["phase_begin"].shape
        M = table["phase_b"].shape[2]
        return PhaseTable(P, M, _ptr(table["nphases"], torch.int32, (B,), "nphases"),
                          _ptr(table["phase_begin"], torch.float64, (B, P), "phase_begin"),
                          _ptr(table["phase_end"], torch.float64, (B, P), "phase_end"),
                          _ptr(table["phase_A"], torch.float64, (B, P, M, 2), "phase_A"),
                          _ptr(table["phase_b"], torch.float64, (B, P, M), "phase_b"),
                          _ptr(table["phase_nf"], torch.int32, (B, P), "phase_nf"),
                          _ptr(table["phase_ref"], torch.float64, (B, P, 2), "phase_ref"))

    def dcm_mpc_solve_phased(self, table, start, xi_init, omega, params=None, warm=None,
                             out=None, window=None, lambda_out=False, stream=None):
        """blf_dcm_mpc_solve_phased: dcm_phase_expand(table, start, params.dt, N) followed by
        dcm_mpc_solve on that window, fused (same results bit for bit, N <= 128).
        omega [B, N] or a row-strided view [B, N] of a longer [B, L] array (stride(1) == 1).
        window: scratch dict (omega, xi_ref, vrp_ref, A, b, nfacets) of the window's shapes, kept
        in out["window"] (allocated once when absent)."""
        torch = _torch()
        B, N = omega.shape
        M = table["phase_b"].shape[2]
        p = params if params is not None else default_params(N, max_facets=M)
        if p.horizon != N or p.max_facets != M:
            raise ValueError("params.horizon / max_facets do not match omega / the phase table")
        if omega.device.type != "cuda" or omega.dtype != torch.float64 or omega.stride(1) != 1:
            raise ValueError("omega must be a float64 device tensor with unit column stride")
        ostride = omega.stride(0) if B > 1 else N
        dev = omega.device
        if out is None:
            out = dict(xi=torch.empty((B, N + 1, 2), dtype=torch.float64, device=dev),
                       vrp=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
                       status=torch.empty((B,), dtype=torch.int32, device=dev),
                       iters=torch.empty((B,), dtype=torch.int32, device=dev),
                       polished=torch.empty((B,), dtype=torch.int32, device=dev),
                       passes=torch.empty((B,), dtype=torch.int32, device=dev))
        if window is None:
            window = out.get("window")
        if window is None:
            window = dict(omega=torch.empty((B, N), dtype=torch.float64, device=dev),
                          xi_ref=torch.empty((B, N + 1, 2), dtype=torch.float64, device=dev),
                          vrp_ref=torch.empty((B, N, 2), dtype=torch.float64, device=dev),
                          A=torch.empty((B, N, M, 2), dtype=torch.float64, device=dev),
                          b=torch.empty((B, N, M), dtype=torch.float64, device=dev),
                          nfacets=torch.empty((B, N), dtype=torch.int32, device=dev))
            out["window"] = window
        win = DcmMpcWindow(_ptr(window["omega"], torch.float64, (B, N), "window omega"),
                           _ptr(window["xi_ref"], torch.float64, (B, N + 1, 2), "window xi_ref"),
                           _ptr(window["vrp_ref"], torch.float64, (B, N, 2), "window vrp_ref"),
                           _ptr(window["A"], torch.float64, (B, N, M, 2), "window A"),
                           _ptr(window["b"], torch.float64, (B, N, M), "window b"),
                           _ptr(window["nfacets"], torch.int32, (B, N), "window nfacets"))
        tb = self._phase_table_struct(table)
        so = DcmMpcSolution(
            _ptr(out["xi"], torch.float64, (B, N + 1, 2), "xi"),
            _ptr(out["vrp"], torch.float64, (B, N, 2), "vrp"),
            _ptr(out["status"], torch.int32, (B,), "status"),
            _ptr(out["iters"], torch.int32, (B,), "iters"),
            _ptr(out["polished"], torch.int32, (B,), "polished") if "polished" in out else None,
            _ptr(out["passes"], torch.int32, (B,), "passes") if "passes" in out else None)
        ws = None
        if warm is not None:
            ws = _warm_start(warm, B, N, M)
        lam_ptr = None
        if lambda_out:
            if "lam" not in out:
                out["lam"] = torch.empty((B, N, M), dtype=torch.float64, device=dev)
            lam_ptr = _ptr(out["lam"], torch.float64, (B, N, M), "lam")
        self._keep = (tb, so, ws, win)
        args = (self._h, ctypes.byref(p), ctypes.byref(tb), int(start),
                _ptr(xi_init, torch.float64, (B, 2), "xi_init"), _vp(omega.data_ptr()), ostride,
                ctypes.byref(ws) if ws is not None else None, B, ctypes.byref(win), ctypes.byref(so),
                lam_ptr)
        _check(lib().blf_dcm_mpc_solve_phased(*args, _stream(stream)))
        return out

    # --- C3 pipeline: corner sets -> polygons (device hull) -> QP arrays ---
    def assemble_constraints(self, corners, ncorners, max_facets=8, stream=None):
        """corners [B, N+1, P, 2], ncorners [B, N+1] (device) -> A [B,N,M,2], b [B,N,M],
        nfacets [B,N] for knots 0..N-1 via blf_hull2d_hrep."""
        torch = _torch()
        B, N1, P, _ = corners.shape
        N = N1 - 1
        pts = corners[:, :N].reshape(B * N, P, 2).contiguous()
        npts = ncorners[:, :N].reshape(B * N).contiguous()
        A, b, nf = self.hull2d_hrep(pts, npts, max_facets, stream=stream)
        return A.view(B, N, max_facets, 2), b.view(B, N, max_facets), nf.view(B, N)

    # ---- config 5: contact model and floating-base kinematics ---------------------------------
    def _contact_inputs(self, params, twist, pose, null_pose):
        torch = _torch()
        B = twist.shape[0]
        shared = params.dim() == 1
        pp = _ptr(params, torch.float64, (4,) if shared else (B, 4), "params")
        return (B, shared, pp, _ptr(twist, torch.float64, (B, 6), "twist"),
                _ptr(pose, torch.float64, (B, 12), "pose"),
                _ptr(null_pose, torch.float64, (B, 12), "null_pose"))

    def contact_model_eval(self, params, twist, pose, null_pose,
                           outputs=("wrench", "autonomous", "control", "regressor"), stream=None):
        """ContinuousContactModel for a batch: params [B,4] or [4] (L, W, k, b), twist [B,6],
        pose / null_pose [B,12] = (p, R row-major).  Returns the requested outputs."""
        torch = _torch()
        B, shared, pp, tw, ps, ns = self._contact_inputs(params, twist, pose, null_pose)
        shapes = dict(wrench=(B, 6), autonomous=(B, 6), control=(B, 6, 6), regressor=(B, 6, 2))
        out = {k: torch.empty(shapes[k], dtype=torch.float64, device=twist.device) for k in outputs}
        ptrs = [ctypes.c_void_p(out[k].data_ptr()) if k in out else None
                for k in ("wrench", "autonomous", "control", "regressor")]
        _check(lib().blf_contact_model_eval(self._h, pp, 1 if shared else 0, tw, ps, ns, B,
                                            *ptrs, _stream(stream)))
        return out

    def contact_point_wrench(self, params, twist, pose, null_pose, points, stream=None):
        """Force / torque at points [B,Q,2] of each contact surface -> ([B,Q,3], [B,Q,3])."""
        torch = _torch()
        B, shared, pp, tw, ps, ns = self._contact_inputs(params, twist, pose, null_pose)
        Q = points.shape[1]
        f = torch.empty((B, Q, 3), dtype=torch.float64, device=twist.device)
        t = torch.empty_like(f)
        _check(lib().blf_contact_point_wrench(
            self._h, pp, 1 if shared else 0, tw, ps, ns, B,
            _ptr(points, torch.float64, (B, Q, 2), "points"), Q, ctypes.c_void_p(f.data_ptr()),
            ctypes.c_void_p(t.data_ptr()), _stream(stream)))
        return f, t

    def fbk_dynamics(self, rho, rot, twist, joint_vel, stream=None):
        """FloatingBaseSystemKinematics::dynamics: rot [B,3,3], twist [B,6], joint_vel [B,n]."""
        torch = _torch()
        B, n = joint_vel.shape
        dp = torch.empty((B, 3), dtype=torch.float64, device=twist.device)
        dR = torch.empty((B, 3, 3), dtype=torch.float64, device=twist.device)
        dq = torch.empty((B, n), dtype=torch.float64, device=twist.device)
        _check(lib().blf_fbk_dynamics(
            self._h, n, float(rho), _ptr(rot, torch.float64, (B, 3, 3), "rot"),
            _ptr(twist, torch.float64, (B, 6), "twist"),
            _ptr(joint_vel, torch.float64, (B, n), "joint_vel") if n else None,
            ctypes.c_void_p(dp.data_ptr()), ctypes.c_void_p(dR.data_ptr()),
            ctypes.c_void_p(dq.data_ptr()) if n else None, B, _stream(stream)))
        return dp, dR, dq

    def fbk_euler_integrate(self, rho, pos, rot, joints, twist, joint_vel, t0, t1, dT,
                            stream=None):
        """ForwardEuler<FloatingBaseSystemKinematics>::integrate in place on pos [B,3],
        rot [B,3,3], joints [B,n] with constant twist [B,6] and joint_vel [B,n]."""
        torch = _torch()
        B, n = joints.shape
        _check(lib().blf_fbk_euler_integrate(
            self._h, n, float(rho), _ptr(pos, torch.float64, (B, 3), "pos"),
            _ptr(rot, torch.float64, (B, 3, 3), "rot"),
            _ptr(joints, torch.float64, (B, n), "joints") if n else None,
            _ptr(twist, torch.float64, (B, 6), "twist"),
            _ptr(joint_vel, torch.float64, (B, n), "joint_vel") if n else None,
            B, float(t0), float(t1), float(dT), _stream(stream)))
        return pos, rot, joints

    # ---- config 5: floating-base dynamics ------------------------------------------------------
    def fb_model(self, model, rho=0.01, gravity=(0.0, 0.0, -9.81)):
        """Upload a blf/robot.py model; returns an object keeping the device arrays alive."""
        torch = _torch()
        dev = torch.device("cuda", self.device)

        class _M:
            pass
        dm = _M()
        f64 = lambda a: torch.as_tensor(a, dtype=torch.float64).contiguous().to(dev)
        i32 = lambda a: torch.as_tensor(a, dtype=torch.int32).contiguous().to(dev)
        dm.t = dict(parent=i32(model["parent"]), joint_origin=f64(model["joint_origin"]),
                    joint_rot=f64(model["joint_rot"]), joint_axis=f64(model["joint_axis"]),
                    link_mass=f64(model["link_mass"]), link_com=f64(model["link_com"]),
                    link_inertia=f64(model["link_inertia"]), frame_link=i32(model["frame_link"]),
                    frame_pose=f64(model["frame_pose"]))
        if model.get("joint_type") is not None:   # absent: every joint revolute (NULL)
            jt = torch.as_tensor(model["joint_type"], dtype=torch.int32)
            if not ((jt == 0) | (jt == 1)).all():
                raise ValueError("joint_type: every entry must be 0 (revolute) or 1 (prismatic); merge fixed "
                                 "joints first (blf.robot.reduce_fixed_joints)")
            dm.t["joint_type"] = i32(jt)
        c = FbModel()
        c.ndof = int(model["n"])
        c.nframes = int(len(model["frame_link"]))
        for k, v in dm.t.items():
            setattr(c, k, _vp(v.data_ptr()))
        for i in range(3):
            c.gravity[i] = gravity[i]
        c.rho = rho
        dm.c = c
        dm.n = c.ndof
        return dm

    def _fb_state(self, st, B, n):
        torch = _torch()
        shapes = dict(base_vel=(B, 6), joint_vel=(B, n), base_pos=(B, 3), base_rot=(B, 3, 3),
                      joint_pos=(B, n))
        c = FbState()
        for k in FB_STATE_KEYS:
            setattr(c, k, _ptr(st[k], torch.float64, shapes[k], k))
        return c

    def _fb_contacts(self, contacts, B):
        torch = _torch()
        c = FbContacts()
        if not contacts:
            c.ncontacts = 0
            return c
        C = contacts["frame"].shape[0]
        c.ncontacts = C
        c.frame = _ptr(contacts["frame"], torch.int32, (C,), "frame")
        c.params = _ptr(contacts["params"], torch.float64, (C, 4), "params")
        c.null_pose = _ptr(contacts["null_pose"], torch.float64, (B, C, 12), "null_pose")
        if contacts.get("law") is not None:
            c.law = _ptr(contacts["law"], torch.int32, (C,), "law")
            w = contacts.get("wrench")   # required by the library (checked there)
            c.wrench = _ptr(w, torch.float64, (B, C, 6), "wrench") if w is not None else None
        return c

    def fbd_dynamics(self, dm, state, torque, contacts=None, mass_reg=None, stream=None):
        """FloatingBaseDynamicalSystem::dynamics for a batch.  state: dict of device tensors
        (base_vel [B,6], joint_vel [B,n], base_pos [B,3], base_rot [B,3,3], joint_pos [B,n]);
        torque [B,n]; contacts: dict(frame [C] int32, params [C,4], null_pose [B,C,12]) and
        optionally law [C] int32 (CONTACT_CONTINUOUS / CONTACT_WRENCH) with wrench [B,C,6] (the
        CONTACT_WRENCH contacts' (force, torque), mixed representation at the frame).
        Returns the derivative with the same keys (base_vel -> base acceleration, ...)."""
        torch = _torch()
        B, n = state["joint_pos"].shape
        out = {k: torch.empty_like(state[k]) for k in FB_STATE_KEYS}
        NV = n + 6
        reg = _ptr(mass_reg, torch.float64, (NV, NV), "mass_reg") if mass_reg is not None else None
        st, oc = self._fb_state(state, B, n), self._fb_state(out, B, n)
        ct = self._fb_contacts(contacts, B)
        _check(lib().blf_fbd_dynamics(self._h, ctypes.byref(dm.c), ctypes.byref(st),
                                      _ptr(torque, torch.float64, (B, n), "torque"),
                                      ctypes.byref(ct), reg, B, ctypes.byref(oc),
                                      _stream(stream)))
        return out

    def fbd_euler_integrate(self, dm, state, torque, t0, t1, dT, contacts=None, mass_reg=None,
                            stream=None):
        """ForwardEuler<FloatingBaseDynamicalSystem>::integrate in place on `state`."""
        torch = _torch()
        B, n = state["joint_pos"].shape
        NV = n + 6
        reg = _ptr(mass_reg, torch.float64, (NV, NV), "mass_reg") if mass_reg is not None else None
        st = self._fb_state(state, B, n)
        ct = self._fb_contacts(contacts, B)
        _check(lib().blf_fbd_euler_integrate(self._h, ctypes.byref(dm.c), ctypes.byref(st),
                                             _ptr(torque, torch.float64, (B, n), "torque"),
                                             ctypes.byref(ct), reg, B, float(t0), float(t1),
                                             float(dT), _stream(stream)))
        return state

    def fb_frame_state(self, dm, state, frames, pose=None, twist=None, stream=None):
        """blf_fb_frame_state: world transform pose [B,K,12] = (p, R row-major) and mixed twist
        [B,K,6] = (v, w) of the frames [K] (int32 device tensor) of every system -- the state a
        CONTACT_WRENCH contact model is evaluated at."""
        torch = _torch()
        B, n = state["joint_pos"].shape
        K = frames.shape[0]
        dev = state["joint_pos"].device
        pose = pose if pose is not None else torch.empty((B, K, 12), dtype=torch.float64, device=dev)
        twist = twist if twist is not None else torch.empty((B, K, 6), dtype=torch.float64, device=dev)
        _check(lib().blf_fb_frame_state(self._h, ctypes.byref(dm.c),
                                        ctypes.byref(self._fb_state(state, B, n)), K,
                                        _ptr(frames, torch.int32, (K,), "frames"), B,
                                        _ptr(pose, torch.float64, (B, K, 12), "pose"),
                                        _ptr(twist, torch.float64, (B, K, 6), "twist"),
                                        _stream(stream)))
        return pose, twist

    # ---- config 5: the closed loop's maps ----------------------------------
    def fb_dcm(self, dm, state, omega=None, column=0, com=None, xi=None, stream=None):
        """blf_fb_dcm: centre of mass and its velocity com [B,6] of every system and, when omega
        ([B,K] device tensor) is given, the DCM xi [B,2] = c_xy + cdot_xy / omega[:, column]."""
        torch = _torch()
        B, n = state["joint_pos"].shape
        dev = state["joint_pos"].device
        com = com if com is not None else torch.empty((B, 6), dtype=torch.float64, device=dev)
        optr, ostride = None, 0
        if omega is not None:
            K = omega.shape[1]
            _ptr(omega, torch.float64, (B, K), "omega")
            if not 0 <= column < K:
                raise ValueError(f"omega column {column} outside [0, {K})")
            optr, ostride = _vp(omega.data_ptr() + 8 * column), K
            xi = xi if xi is not None else torch.empty((B, 2), dtype=torch.float64, device=dev)
        elif xi is not None:
            raise ValueError("xi requested without omega")
        _check(lib().blf_fb_dcm(self._h, ctypes.byref(dm.c), ctypes.byref(self._fb_state(state, B, n)),
                                optr, ostride, B, _ptr(com, torch.float64, (B, 6), "com"),
                                _ptr(xi, torch.float64, (B, 2), "xi") if xi is not None else None,
                                _stream(stream)))
        return com, xi

    def posture_law(self, q_nominal, lean):
        """Upload a blf_posture_law: q_nominal [n], lean [n,2] (host arrays)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)

        class _L:
            pass
        law = _L()
        f64 = lambda a: torch.as_tensor(a, dtype=torch.float64).contiguous().to(dev)
        law.t = dict(q_nominal=f64(q_nominal), lean=f64(lean))
        n = law.t["q_nominal"].shape[0]
        if law.t["lean"].shape != (n, 2):
            raise ValueError("posture law: q_nominal [n] and lean [n,2]")
        c = PostureLaw()
        c.ndof = n
        c.q_nominal, c.lean = _vp(law.t["q_nominal"].data_ptr()), _vp(law.t["lean"].data_ptr())
        law.c = c
        return law

    def posture_reference(self, law, com, vrp, q_ref=None, stream=None):
        """blf_dcm_posture_reference: joint references [B,n] from the plan's first VRP (vrp
        [B,N,2], a blf_dcm_mpc_solve output) and the centre of mass com [B,6] (fb_dcm)."""
        torch = _torch()
        B, N = vrp.shape[0], vrp.shape[1]
        n = law.c.ndof
        q_ref = q_ref if q_ref is not None else torch.empty((B, n), dtype=torch.float64,
                                                            device=vrp.device)
        args = (self._h, ctypes.byref(law.c), _ptr(com, torch.float64, (B, 6), "com"),
                _ptr(vrp, torch.float64, (B, N, 2), "vrp"), 2 * N, B,
                _ptr(q_ref, torch.float64, (B, n), "q_ref"))
        _check(lib().blf_dcm_posture_reference(*args, _stream(stream)))
        return q_ref

    def joint_impedance(self, kp, kd):
        """Device copies of the impedance gains kp, kd [n] (host arrays)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        f64 = lambda a: torch.as_tensor(a, dtype=torch.float64).contiguous().to(dev)
        return dict(kp=f64(kp), kd=f64(kd))

    def fbd_euler_integrate_impedance(self, dm, state, impedance, q_ref, t0, t1, dT, contacts=None,
                                      mass_reg=None, stream=None):
        """blf_fbd_euler_integrate_impedance in place on `state`: the control input of every
        Euler step is tau = kp (q_ref - q) - kd qdot (impedance: joint_impedance())."""
        torch = _torch()
        B, n = state["joint_pos"].shape
        NV = n + 6
        reg = _ptr(mass_reg, torch.float64, (NV, NV), "mass_reg") if mass_reg is not None else None
        imp = JointImpedance()
        imp.ndof = n
        imp.kp = _ptr(impedance["kp"], torch.float64, (n,), "kp")
        imp.kd = _ptr(impedance["kd"], torch.float64, (n,), "kd")
        imp.q_ref = _ptr(q_ref, torch.float64, (B, n), "q_ref")
        args = (self._h, ctypes.byref(dm.c), ctypes.byref(self._fb_state(state, B, n)), ctypes.byref(imp),
                ctypes.byref(self._fb_contacts(contacts, B)), reg, B, float(t0), float(t1), float(dT))
        _check(lib().blf_fbd_euler_integrate_impedance(*args, _stream(stream)))
        return state
