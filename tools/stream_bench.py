"""HBM roofline of the streaming kernels (the 40 % HBM bar applies to these):
dcm_rollout, hull2d_hrep, quintic_eval, contact_model_eval, fbk_euler (1 step), phase_expand on
large batches.
achieved = algorithmic bytes / median kernel time (HIP events).
  python tools/stream_bench.py [--out gpurun_out/stream.json]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))
from blf import native  # noqa: E402

PEAK = 8000.0   # GB/s


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    h = native.Handle(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.rand(*s, dtype=torch.float64, device=dev, generator=g)
    lines = []

    def report(name, nbytes, ms, units, unit_name):
        gbs = nbytes / (ms * 1e-3) / 1e9
        lines.append(dict(kernel=name, ms=ms, algorithmic_bytes=nbytes, achieved_gbs=gbs,
                          peak_gbs=PEAK, frac=gbs / PEAK, units=units, unit=unit_name))
        print(json.dumps(lines[-1]), flush=True)

    # dcm_rollout: 40 B per problem-knot (+16 B xi0 per problem)
    B, N = 262144, 100
    xi0, om, vrp = rnd(B, 2), rnd(B, N) * 4 + 3, rnd(B, N, 2)
    out = torch.empty(B, N + 1, 2, dtype=torch.float64, device=dev)
    ms = timed(lambda: h.dcm_euler_rollout(xi0, om, vrp, 0.02, out=out))
    report("dcm_rollout_rows_kernel", B * (N * 40 + 16 + 16), ms, B * N, "problem-knots")
    del xi0, om, vrp, out
    # hull2d_hrep: 8 points per polygon, M = 8 rows
    P, M = 2 * 1024 * 1024, 8
    ang = rnd(P, 8) * 6.283
    pts = torch.stack([torch.cos(ang), torch.sin(ang)], dim=-1).contiguous()
    npts = torch.full((P,), 8, dtype=torch.int32, device=dev)
    ms = timed(lambda: h.hull2d_hrep(pts, npts, M))
    report("hull2d_kernel", P * (16 * 8 + 4 + 24 * M + 4), ms, P, "polygons")
    del pts, npts, ang
    # quintic_eval: S splines of 3 knots, 3 axes, Q queries
    S, Q = 1024 * 1024, 32
    kt = torch.cumsum(rnd(S, 3) + 0.1, dim=1).contiguous()
    kp = rnd(S, 3, 3, 3)
    co = h.quintic_fit(kt, kp)
    tq = (kt[:, :1] + (kt[:, 2:] - kt[:, :1]) * rnd(S, Q)).contiguous()
    ms = timed(lambda: h.quintic_eval(kt, co, tq))
    report("quintic_eval_kernel", S * (Q * (8 + 72 + 4) + 3 * 8 + 2 * 3 * 6 * 8), ms, S * Q,
           "queries")
    del kt, kp, co, tq
    # what the memory system gives a plain stream on this box: torch's write-only fill and copy
    # of 3 GiB (reference lines for the write-dominated kernels above, not library kernels)
    big = torch.empty(3 * 2 ** 27, dtype=torch.float64, device=dev)
    ms = timed(lambda: big.fill_(1.0))
    report("ref:torch_fill", big.numel() * 8, ms, big.numel(), "doubles")
    half = big[: big.numel() // 2]
    other = big[big.numel() // 2:]
    ms = timed(lambda: other.copy_(half))
    report("ref:torch_copy", half.numel() * 16, ms, half.numel(), "doubles")
    del big, half, other
    # contact_model_eval: all four outputs
    C = 4 * 1024 * 1024
    prm = torch.tensor([0.12, 0.09, 2000.0, 100.0], dtype=torch.float64, device=dev)
    tw, pose, null = rnd(C, 6), rnd(C, 12), rnd(C, 12)
    ms = timed(lambda: h.contact_model_eval(prm, tw, pose, null))
    report("contact_eval_kernel", C * 8 * (6 + 12 + 12 + 6 + 6 + 36 + 12), ms, C, "contacts")
    ms = timed(lambda: h.contact_model_eval(prm, tw, pose, null, outputs=("wrench",)))
    report("contact_eval_kernel[wrench]", C * 8 * (6 + 12 + 12 + 6), ms, C, "contacts")
    del tw, pose, null
    # fbk dynamics: n = 24
    F, n = 2 * 1024 * 1024, 24
    R, tw, sd = rnd(F, 3, 3), rnd(F, 6), rnd(F, n)
    ms = timed(lambda: h.fbk_dynamics(0.01, R, tw, sd))
    report("fbk_dynamics_kernel", F * 8 * ((9 + 6 + n) + (3 + 9 + n)), ms, F, "systems")
    pos, jt = rnd(F, 3), rnd(F, n)
    ms = timed(lambda: h.fbk_euler_integrate(0.01, pos, R, jt, tw, sd, 0.0, 0.001, 0.001))
    report("fbk_euler_kernel[1 step]", F * 8 * (2 * (3 + 9 + n) + 6 + n), ms, F, "systems")
    del R, tw, sd, pos, jt
    # dcm_phase_expand: 32768 plans of 13 phases, horizon-100 windows
    from blf import problems as P
    Bq, N = 32768, 100
    prob = P.make_batch(Bq, horizon=N + 8, n_footsteps=8, seed=P.SEED)
    t = lambda k: torch.from_numpy(prob[k]).to(dev)
    table = h.phase_table(t("nphases"), t("phase_begin"), t("phase_end"), t("phase_corners"),
                          t("phase_ncorners"), ref=t("phase_ref"))
    Pn, M = table["phase_begin"].shape[1], 8
    w = h.dcm_phase_expand(table, 3, prob["dt"], N)
    ms = timed(lambda: h.dcm_phase_expand(table, 3, prob["dt"], N, out=w))
    report("phase_expand_kernel", Bq * (4 + Pn * (16 + 24 * M + 4 + 16) + N * (24 * M + 4 + 16)
                                        + 16 * (N + 1)), ms, Bq, "windows")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(lines, f, indent=1)


if __name__ == "__main__":
    main()
