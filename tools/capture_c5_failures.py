"""Runs bench.py's configs[4] loop on the device (one group, rank 0's shard, 3 + 20 periods) and
writes every window whose solve did not end at status 0 -- with the inputs of its warm solve, in
tests/golden/c5_*_windows.npz's layout -- to gpurun_out/c5_device_failures.npz (a tool: the
windows then become a fixture the oracle and the device are checked on)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))
from blf import closed_loop as DL   # noqa: E402
from blf import native               # noqa: E402
from blf import problems as P        # noqa: E402
from blf import robot                # noqa: E402


INTS = ("nfacets", "prev_status", "robot", "period", "status", "iters")


def main():
    B, N, periods = 16384, 100, 23
    model = robot.humanoid24()
    plan = P.make_batch(B, horizon=N + periods, n_footsteps=8, seed=P.SEED, start=0, first_ds=periods + 10)
    st = robot.standing_states(model, B, seed=1000)
    h = native.Handle(0)
    loop = DL.ClosedLoop(h, model, plan, st, horizon=N)
    keep = {k: [] for k in ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets", "vrp_ws", "lam_ws",
                            "prev_status", "robot", "period", "status", "iters")}
    for s in range(periods):
        prev = loop.prev
        out = loop.period()
        torch.cuda.synchronize()
        stat = out["status"].cpu().numpy()
        bad = np.nonzero(stat != 0)[0]
        print(f"period {s}: {int((out['iters'] > 0).sum())} windows in the interior point kernel, "
              f"{len(bad)} unsolved", flush=True)
        w = out["window"]
        for i in bad:
            keep["xi_init"].append(loop.xi[i].cpu().numpy())
            for k in ("omega", "xi_ref", "vrp_ref", "A", "b", "nfacets"):
                keep[k].append(w[k][i].cpu().numpy())
            keep["vrp_ws"].append(prev["vrp"][i].cpu().numpy())
            keep["lam_ws"].append(prev["lam"][i].cpu().numpy())
            # the status the warm solve was given (the loop's cold-after-hand-over rule applied)
            keep["prev_status"].append(int((loop.warm_status if loop.cold_after_handover else prev["status"])[i]))
            keep["robot"].append(int(i))
            keep["period"].append(s)
            keep["status"].append(int(stat[i]))
            keep["iters"].append(int(out["iters"][i]))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    if keep["robot"]:
        np.savez(os.path.join(ROOT, "gpurun_out", "c5_device_failures.npz"),
                 **{k: np.asarray(v, dtype=np.int32 if k in INTS else None) for k, v in keep.items()})
    print("captured", len(keep["robot"]))


if __name__ == "__main__":
    main()
