"""Diagnostics: device time of the warm solve of the committed hard c5 windows
(tests/golden/c5_hard_windows.npz): all 128 at once, and the slowest single window alone, each
10 launches after a warm-up, HIP events around the launch.  Run under rocprofv3 --kernel-trace
--stats for the per-kernel split (active-set warm kernel / interior point kernel)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))
from blf import native  # noqa: E402

KEYS = ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")


def run(h, d, sel, reps=10):
    dev = {k: torch.from_numpy(np.ascontiguousarray(d[k][sel])).cuda() for k in KEYS}
    N = dev["omega"].shape[1]
    prm = native.default_params(N, tol_polish=1e-4)
    warm = dict(vrp=torch.from_numpy(np.ascontiguousarray(d["vrp_ws"][sel])).cuda(),
                lam=torch.from_numpy(np.ascontiguousarray(d["lam_ws"][sel])).cuda(), shift=1, floor=1e-3,
                status=torch.from_numpy(np.ascontiguousarray(d["prev_status"][sel])).cuda())
    out = h.dcm_mpc_solve(dev, prm, warm=warm)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out = h.dcm_mpc_solve(dev, prm, warm=warm, out=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, out["iters"].cpu().numpy()


def main():
    d = dict(np.load(os.path.join(ROOT, "tests", "golden", "c5_hard_windows.npz")))
    h = native.Handle(0)
    ms, it = run(h, d, slice(None))
    print(f"all {len(it)} hard windows: {ms:.3f} ms per warm solve, IPM iterations mean {it.mean():.1f} max {it.max()}")
    j = int(np.argmax(it))
    ms1, it1 = run(h, d, slice(j, j + 1))
    print(f"window {j} alone ({it1[0]} IPM iterations): {ms1:.3f} ms per warm solve")
    ms0, it0 = run(h, d, slice(int(np.argmin(it)), int(np.argmin(it)) + 1))
    print(f"window {int(np.argmin(it))} alone ({it0[0]} IPM iterations): {ms0:.3f} ms")
    L = native.lib()
    if hasattr(L, "blf_debug_stamps"):   # the stamp build: the IPM kernel's phases, window j alone
        import ctypes
        buf = (ctypes.c_ulonglong * 16)()
        L.blf_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.blf_debug_stamps(ctypes.cast(buf, ctypes.c_void_p), 1)
        run(h, d, slice(j, j + 1), reps=1)
        L.blf_debug_stamps(ctypes.cast(buf, ctypes.c_void_p), 0)
        names = ["total", "factor", "solve", "iterations", "residuals", "W-phase", "predictor solve",
                 "step+update", "polish", "polish attempts", "loads", "LQ step", "start point",
                 "polish projection+residuals", "polish Riccati", "polish solve"]
        print("stamps (window %d, 2 launches, thread 0): " % j +
              ", ".join(f"{n} {v}" for n, v in zip(names, list(buf))))


if __name__ == "__main__":
    main()
