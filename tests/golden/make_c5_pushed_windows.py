"""Generates tests/golden/c5_pushed_windows.npz: the receding-horizon windows of PUSHED robots that
the round-5 solver ended unsolved ("what's missing" 1 / "next" 2).

The scenario is tests/test_gpu_closed_loop.py::test_closed_loop_stage2_list_bitwise: 160 robots of
the config-5 closed loop (8-footstep plans, standing start, seed 3), every fifth one pushed with a
lateral base velocity of +1.2 m/s, 4 control periods, run on the CPU through oracle/closed_loop.py
(OracleLoop, compiled).  Every pushed robot is uncapturable: its DCM runs to 10^2-10^3 m over the
horizon, the costates reach 1e10 and the multipliers 1e8-1e9.  With the round-5 oracle (build it
from `git show 1ccd666:oracle/<file>` and point BLF_ORACLE_LIB at it) 24-27 windows per period
ended at MAX_ITER or NUMERICAL; these QPs are feasible and strictly convex (the only inequalities
are the support polygons on r_k), so each has a unique optimum.  Kept: every window whose solve did
not end at status 0, with the inputs of its warm solve (the period-0 windows are cold: zero warm
start, prev_status 1).

    BLF_ORACLE_LIB=/tmp/liboracle_r05.so python tests/golden/make_c5_pushed_windows.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import closed_loop as CL            # noqa: E402
from blf import closed_loop as DL   # noqa: E402
from blf import problems as P       # noqa: E402
from blf import robot               # noqa: E402

KEYS = ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")
INTS = ("nfacets", "prev_status", "robot", "period", "status", "iters")


def main(B=160, periods=4, N=100, M=8):
    model = robot.humanoid24()
    plan = P.make_batch(B, horizon=N + periods, n_footsteps=8, seed=P.SEED, first_ds=periods + 10)
    st = robot.standing_states(model, B, seed=3)
    st["base_vel"][::5, 1] += 1.2
    loop = CL.OracleLoop(model, plan, st, robot.sole_null_poses(model, st), robot.posture_law_arrays(model),
                         DL.CONTACT_PARAMS, horizon=N, compiled=True)
    keep = {k: [] for k in KEYS + ("vrp_ws", "lam_ws") + INTS[1:]}
    for s in range(periods):
        out = loop.period()
        w = loop.last_window
        bad = np.nonzero(out["status"] != 0)[0]
        print(f"period {s}: {len(bad)} unsolved", flush=True)
        for i in bad:
            for k in KEYS:
                keep[k].append(np.asarray(w[k][i]))
            keep["vrp_ws"].append(np.zeros((N, 2)) if w["vrp_ws"] is None else w["vrp_ws"][i])
            keep["lam_ws"].append(np.zeros((N, M)) if w["lam_ws"] is None else w["lam_ws"][i])
            keep["prev_status"].append(1 if w["prev_status"] is None else int(w["prev_status"][i]))
            keep["robot"].append(int(i))
            keep["period"].append(s)
            keep["status"].append(int(out["status"][i]))
            keep["iters"].append(int(out["iters"][i]))
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c5_pushed_windows.npz")
    np.savez_compressed(out, **{k: np.asarray(v, dtype=np.int32 if k in INTS else np.float64)
                                for k, v in keep.items()})
    print("kept", len(keep["robot"]), "->", out)


if __name__ == "__main__":
    main()
