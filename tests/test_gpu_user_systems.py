"""ForwardEuler<UserSystem> on the device (include/blf/forward_euler_device.h): the reference's
DynamicalSystem::dynamics override (DynamicalSystem.h:98) integrated by ForwardEuler.tpp:18-49
over FixedStepIntegrator.tpp:21-72's schedule, for systems the user states as __device__ code.

* UserLti<3,2> / <8,8> (bipedal-locomotion-framework_amd/host/tests/user_systems.hip) restates
  LinearTimeInvariantSystem as a user system: bit for bit the library's blf_lti_euler_integrate,
  which the oracle pins (tests/test_gpu_kernels.py).
* ForcedOscillator (forcing u t^2, cubic spring) uses the time argument, including the stale
  currentTime of the last step (FixedStepIntegrator.tpp:53-64): bit for bit a plain-Python
  restatement of the reference loop (IEEE doubles, no FMA; the device TU is -ffp-contract=off).
* blf_step_schedule (the C ABI's schedule) against the reference loop and its error codes.
"""
import ctypes
import math
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTLIB = os.path.join(ROOT, "bipedal-locomotion-framework_amd", "lib", "libblf_usersys_test.so")


def _lib():
    L = ctypes.CDLL(TESTLIB)
    for name in ("blf_test_user_lti3x2", "blf_test_user_lti8x8", "blf_test_user_forced_oscillator"):
        f = getattr(L, name)
        f.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                      ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
        f.restype = ctypes.c_int32
    return L


def _schedule(t0, T, dT):
    """FixedStepIntegrator::integrate's loop (FixedStepIntegrator.tpp:48-64): (time, step) pairs."""
    it = int(math.ceil((T - t0) / dT))
    steps, cur = [], t0
    for i in range(it - 1):
        cur = t0 + dT * i
        steps.append((cur, dT))
    steps.append((cur, T - cur))
    return steps


def test_step_schedule_matches_reference_loop():
    from blf import native
    L = native.lib()
    f = L.blf_step_schedule
    f.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_int32),
                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    f.restype = ctypes.c_int32
    it, dl, tl = ctypes.c_int32(), ctypes.c_double(), ctypes.c_double()
    for t0, T, dT in ((0.0, 0.02, 0.001), (0.0, 0.019, 0.001), (0.3, 1.0, 0.07), (0.0, 0.0005, 0.001),
                      (1.0, 1.25, 0.1), (-2.0, 3.0, 0.3)):
        assert f(t0, T, dT, ctypes.byref(it), ctypes.byref(dl), ctypes.byref(tl)) == 0
        ref = _schedule(t0, T, dT)
        assert it.value == len(ref)
        assert (tl.value, dl.value) == ref[-1]
    assert f(1.0, 0.5, 0.1, ctypes.byref(it), ctypes.byref(dl), ctypes.byref(tl)) == 4   # BLF_ERR_TIME_INTERVAL
    assert f(0.0, 1.0, 0.0, ctypes.byref(it), ctypes.byref(dl), ctypes.byref(tl)) == 4
    assert f(0.5, 0.5, 0.1, ctypes.byref(it), ctypes.byref(dl), ctypes.byref(tl)) == 5   # BLF_ERR_EMPTY_INTERVAL
    assert f(0.0, 1.0, 0.1, None, ctypes.byref(dl), ctypes.byref(tl)) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,B,shared", [(3, 2, 1000, False), (3, 2, 257, True), (8, 8, 300, False)])
def test_user_lti_matches_library_lti(handle, n, m, B, shared):
    import torch
    rng = np.random.default_rng(n * 100 + B)
    A = rng.normal(scale=0.5, size=(1 if shared else B, n, n))
    Bm = rng.normal(size=(1 if shared else B, n, m))
    u = rng.normal(size=(B, m))
    x0 = rng.normal(size=(B, n))
    params = np.concatenate([A.reshape(A.shape[0], -1), Bm.reshape(Bm.shape[0], -1)], axis=1)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    dp, du, xu = dev(params), dev(u), dev(x0)
    fn = getattr(_lib(), f"blf_test_user_lti{n}x{m}")
    for (t0, T, dT) in ((0.0, 0.037, 0.004), (0.1, 0.3, 0.05)):
        xu = dev(x0)
        assert fn(dp.data_ptr(), int(shared), du.data_ptr(), xu.data_ptr(), B, t0, T, dT, None) == 0
        xl = dev(x0)
        handle.lti_euler_integrate(dev(A[0] if shared else A), dev(Bm[0] if shared else Bm), du, xl, t0, T, dT,
                                   shared=shared)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(xu.cpu().numpy(), xl.cpu().numpy())


def _oscillator_ref(x, u, p, t0, T, dT):
    q, v = float(x[0]), float(x[1])
    k, c, k3 = (float(a) for a in p)
    for t, h in _schedule(t0, T, dT):
        d0 = v
        d1 = ((u * (t * t) - k * q) - c * v) - k3 * (q * q * q)
        q, v = q + d0 * h, v + d1 * h
    return q, v


@pytest.mark.gpu
@pytest.mark.parametrize("t0,T,dT", [(0.0, 0.02, 0.001), (0.25, 1.0, 0.03), (0.0, 0.0007, 0.001)])
def test_user_forced_oscillator_matches_reference_loop(t0, T, dT):
    import torch
    B = 129
    rng = np.random.default_rng(7)
    x0 = rng.normal(size=(B, 2))
    u = rng.normal(size=(B, 1))
    p = np.c_[rng.uniform(1, 50, B), rng.uniform(0, 2, B), rng.uniform(0, 5, B)]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    x = dev(x0)
    assert _lib().blf_test_user_forced_oscillator(dev(p).data_ptr(), 0, dev(u).data_ptr(), x.data_ptr(), B,
                                                  t0, T, dT, None) == 0
    torch.cuda.synchronize()
    got = x.cpu().numpy()
    for i in range(B):
        assert tuple(got[i]) == _oscillator_ref(x0[i], u[i, 0], p[i], t0, T, dT), i


@pytest.mark.gpu
def test_user_system_argument_errors():
    L = _lib()
    assert L.blf_test_user_forced_oscillator(None, 0, None, None, 0, 0.0, 1.0, 0.1, None) == 0      # empty batch
    assert L.blf_test_user_forced_oscillator(None, 0, None, None, 5, 0.0, 1.0, 0.1, None) == 1      # null buffers
    assert L.blf_test_user_forced_oscillator(None, 0, None, None, 5, 1.0, 0.0, 0.1, None) == 4      # t0 > T
    assert L.blf_test_user_forced_oscillator(None, 0, None, None, 5, 1.0, 1.0, 0.1, None) == 5      # t0 == T
