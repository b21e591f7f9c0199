"""Kernel micro-benchmark of blf_dcm_mpc_solve (diagnostics; not the driver's bench.py).

Times the solve on the bench workload with HIP events and, when the loaded library is the
stamp-instrumented diagnostic build (BLF_LIB=.../libblf_stamps.so), prints where thread 0 of the
first 64 workgroups spends its cycles.
  python tools/kbench.py [--batch 4096] [--horizon 100] [--reps 10]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))

import torch  # noqa: E402
from blf import native  # noqa: E402
from blf import problems as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=100)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--footsteps", type=int, default=6)
    ap.add_argument("--tol-polish", type=float, nargs="*", default=[None])
    args = ap.parse_args()
    for tp in args.tol_polish:
        run(args, tp)


def run(args, tol_polish):
    h = native.Handle(0)
    prob = P.make_batch(args.batch, horizon=args.horizon, n_footsteps=args.footsteps, seed=P.SEED)
    d = {k: torch.from_numpy(prob[k]).cuda() for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}
    A, b, nf = h.assemble_constraints(torch.from_numpy(prob["corners"]).cuda(),
                                      torch.from_numpy(prob["ncorners"]).cuda())
    d.update(A=A, b=b, nfacets=nf)
    prm = native.default_params(args.horizon)
    if tol_polish is not None:
        prm.tol_polish = tol_polish
    out = h.dcm_mpc_solve(d, params=prm)
    torch.cuda.synchronize()
    L = native.lib()
    stamps = getattr(L, "blf_debug_stamps", None) if hasattr(L, "blf_debug_stamps") else None
    buf = (ctypes.c_ulonglong * 16)()
    if stamps is not None:
        stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        stamps(ctypes.cast(buf, ctypes.c_void_p), 1)
    as_stamps = getattr(L, "blf_debug_as_stamps", None) if hasattr(L, "blf_debug_as_stamps") else None
    abuf = (ctypes.c_ulonglong * 32)()
    if as_stamps is not None:
        as_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
        as_stamps(ctypes.cast(abuf, ctypes.c_void_p), 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        h.dcm_mpc_solve(d, params=prm, out=out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    print(f"lib={native.LIB_PATH} batch={args.batch} N={args.horizon} tol_polish={prm.tol_polish:g}: "
          f"{ms:.3f} ms/solve, polished {out['polished'].float().mean().item():.3f}, "
          f"{args.batch / ms * 1e3:.0f} QP/s, mean iters {out['iters'].float().mean().item():.2f}, "
          f"status!=0: {int((out['status'] != 0).sum())}")
    if as_stamps is not None:
        as_stamps(ctypes.cast(abuf, ctypes.c_void_p), 0)
        q = min(args.batch, 64) * args.reps
        npass = max(abuf[10], 1)
        print(f"active-set kernel, lane 0 cycles per QP: total {abuf[0] / q:.0f}, staging + knot loads "
              f"{abuf[1] / q:.0f}, LQ step {abuf[2] / q:.0f}, guess {abuf[3] / q:.0f}, outputs "
              f"{abuf[11] / q:.0f}, passes {abuf[10] / q:.2f} per QP")
        print(f"per fp64 pass: setup + residuals {abuf[4] / npass:.0f}, Riccati sweep {abuf[5] / npass:.0f}, "
              f"h {abuf[6] / npass:.0f}, solve {abuf[7] / npass:.0f}, certificate {abuf[8] / npass:.0f}, "
              f"vote + restore {abuf[9] / npass:.0f}")
        if abuf[12]:
            n32 = abuf[12]
            print(f"fp32 passes: {abuf[13] / q:.0f} cycles per QP, {n32 / q:.2f} passes; fp64 passes "
                  f"{abuf[14] / q:.0f} cycles per QP; kernel B total {abuf[15] / q:.0f}")
            print(f"per fp32 pass: setup + residuals {abuf[16] / n32:.0f}, Riccati sweep {abuf[17] / n32:.0f}, "
                  f"h {abuf[18] / n32:.0f}, solve {abuf[19] / n32:.0f}, certificate {abuf[20] / n32:.0f}, "
                  f"vote + restore {abuf[21] / n32:.0f}")
    for tl_name in ("blf_debug_as32_timeline", "blf_debug_as_timeline"):
        tl = getattr(L, tl_name, None) if hasattr(L, tl_name) else None
        if tl is None:
            continue
        import numpy as np
        n = min(args.batch, 65536)
        t = np.zeros((n, 4), dtype=np.uint64)
        tl.argtypes = [ctypes.c_void_p, ctypes.c_int]
        tl(t.ctypes.data, n)
        rt0, rt1 = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
        base = rt0.min()
        s0, s1 = (rt0 - base) / 100.0, (rt1 - base) / 100.0   # us
        clk = (t[:, 3].astype(np.int64) - t[:, 2].astype(np.int64)) / ((rt1 - rt0) / 100.0) / 1e3   # GHz
        life = s1 - s0
        print(f"{tl_name} (last launch, {n} QPs): span {s1.max():.1f} us, wave lifetime mean {life.mean():.1f} "
              f"min {life.min():.1f} max {life.max():.1f} us, shader clock median {np.median(clk):.2f} GHz")
        edges = np.linspace(0, s1.max(), 21)
        res = [int(((s0 <= e) & (s1 > e)).sum()) for e in edges[:-1]]
        print("resident waves at 20 instants:", res)
        print("start times quantiles (us):", np.round(np.quantile(s0, [0, .1, .25, .5, .75, .9, 1]), 1).tolist())
    if stamps is not None and not stamps(ctypes.cast(buf, ctypes.c_void_p), 0) and buf[0]:
        tot, fac, sol, its = buf[0], buf[1], buf[2], max(buf[3], 1)
        res, wph, pred, step = buf[4], buf[5], buf[6], buf[7]
        print(f"thread0 cycles per QP: total {tot / 64 / args.reps:.0f}  per iteration: "
              f"residuals {res / its:.0f}, W-phase {wph / its:.0f}, factor {fac / its:.0f}, "
              f"predictor solve {pred / its:.0f}, ratio+mu_aff+corr-rhs+corr-solve "
              f"{(sol - pred) / its:.0f}, step+update {step / its:.0f}, "
              f"unaccounted {(tot - res - wph - fac - sol - step - buf[8]) / its:.0f} "
              f"(iters counted {its / 64 / args.reps:.2f})")
        if buf[9]:
            print(f"polish: {buf[9] / 64 / args.reps:.2f} attempts per QP, {buf[8] / buf[9]:.0f} cycles "
                  f"per attempt; total per QP split: iterations {(tot - buf[8]) / 64 / args.reps:.0f}, "
                  f"polish {buf[8] / 64 / args.reps:.0f}")
        q = min(args.batch, 64) * args.reps
        print(f"start-up per QP: loads {buf[10] / q:.0f}, LQ step {buf[11] / q:.0f}, "
              f"slacks/multipliers/dual residual {buf[12] / q:.0f}")
        if buf[9]:
            na = buf[9]
            print(f"per polish attempt: projection+residuals {buf[13] / na:.0f}, Riccati sweep "
                  f"{buf[14] / na:.0f}, solve {buf[15] / na:.0f}, h + certificate + vote "
                  f"{(buf[8] - buf[13] - buf[14] - buf[15]) / na:.0f}")

if __name__ == "__main__":
    main()
