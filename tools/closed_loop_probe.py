"""Diagnostics: run the config-5 closed loop (blf.closed_loop) on the device for a number of
periods and print, per period, the QP statuses, IPM iterations, the DCM spread and the base
heights.  python tools/closed_loop_probe.py [--batch 16384] [--periods 25] [--spread 0.05]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))

import torch  # noqa: E402
from blf import closed_loop as DL, native, problems as P, robot as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--periods", type=int, default=25)
    ap.add_argument("--spread", type=float, default=0.05)
    ap.add_argument("--vel", type=float, default=0.05)
    args = ap.parse_args()
    h = native.Handle(0)
    m = R.humanoid24()
    B, S = args.batch, args.periods
    plan = P.make_batch(B, horizon=100 + S, n_footsteps=8, seed=P.SEED, first_ds=S + 10)
    st = R.standing_states(m, B, seed=3, spread=args.spread, vel=args.vel)
    loop = DL.ClosedLoop(h, m, plan, st)
    t0 = time.perf_counter()
    for s in range(S):
        out = loop.period()
        torch.cuda.synchronize()
        stat = torch.bincount(out["status"].to(torch.int64), minlength=4).tolist()
        xi = loop.xi
        z = loop.state["base_pos"][:, 2]
        print(f"period {s}: status {stat} iters max {int(out['iters'].max())} mean "
              f"{float(out['iters'].float().mean()):.3f} |xi| max {float(xi.abs().max()):.3f} "
              f"z [{float(z.min()):.3f}, {float(z.max()):.3f}] finite "
              f"{bool(all(torch.isfinite(v).all() for v in loop.state.values()))}", flush=True)
    print(f"{(time.perf_counter() - t0) / S * 1e3:.2f} ms per period (synchronised every period)")


if __name__ == "__main__":
    main()
