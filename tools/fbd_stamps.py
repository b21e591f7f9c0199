"""Per-phase cycles of fbd_eval (lane 0, first 64 systems) from the stamp build:
  BLF_LIB=bipedal-locomotion-framework_amd/lib/libblf_stamps.so python tools/fbd_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))
from blf import native, robot  # noqa: E402

# the articulated-body solve (the default without mass_reg) stamps slots 4-7 as its inward sweep,
# base solve, outward sweep and the whole solve; the factorization path as named in brackets
PHASES = ["joint rot + depth", "forward kinematics", "per-link spatial", "contacts",
          "ABA inward (subtree sums)", "ABA base (columns + rhs)", "ABA outward (mass matrix)",
          "ABA whole (cholesky)", "(substitution)", "total"]


def main():
    h = native.Handle(0)
    L = native.lib()
    B = 16384
    model = robot.humanoid24()
    st = robot.random_states(model, B, seed=9)
    dm = h.fb_model(model)
    d = lambda a, t=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=t).cuda()
    dst = {k: d(st[k]) for k in native.FB_STATE_KEYS}
    null = np.zeros((B, 2, 12))
    null[:, :, 3:] = np.eye(3).reshape(-1)
    ct = dict(frame=d(np.array([0, 1]), torch.int32), params=d(np.array([[0.12, 0.09, 3e4, 300.0]] * 2)),
              null_pose=d(null))
    tau = d(st["joint_torque"])
    f = L.blf_debug_fbd_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 12)()
    h.fbd_dynamics(dm, dst, tau, contacts=ct)
    torch.cuda.synchronize()
    f(ctypes.cast(buf, ctypes.c_void_p), 1)
    reps = 5
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        h.fbd_dynamics(dm, dst, tau, contacts=ct)
    e1.record()
    torch.cuda.synchronize()
    f(ctypes.cast(buf, ctypes.c_void_p), 0)
    evals = 64 * reps
    print(f"fbd_dynamics B={B}: {e0.elapsed_time(e1) / reps:.3f} ms per launch")
    for i, name in enumerate(PHASES):
        print(f"  {name:22s} {buf[i] / evals:10.0f} cycles per eval")


if __name__ == "__main__":
    main()
