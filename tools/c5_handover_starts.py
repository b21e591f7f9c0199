"""The windows of bench.py's configs[4] loop that the warm active-set kernel hands over to the
interior point kernel (iters > 0), captured over 3 + 20 periods of one group (rank 0's shard), and
solved again on the device from their warm start and from a cold start: per period the slowest
window's interior point iterations (the stage-2 kernel's length on the loop's critical path).
A tool: python tools/c5_handover_starts.py -> gpurun_out/c5_handover_starts.npz + a summary."""
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


def main():
    B, N, periods = 16384, 100, 23
    model = robot.humanoid24()
    plan = P.make_batch(B, horizon=N + periods, n_footsteps=8, seed=P.SEED, start=0, first_ds=periods + 10)
    st = robot.standing_states(model, B, seed=1000)
    h = native.Handle(0)
    loop = DL.ClosedLoop(h, model, plan, st, horizon=N)
    keep = {k: [] for k in ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets", "vrp_ws", "lam_ws",
                            "prev_status", "period", "iters")}
    for s in range(periods):
        prev = loop.prev
        out = loop.period()
        xi0 = loop.xi   # this period's initial DCMs (blf_fb_dcm at the period's start)
        torch.cuda.synchronize()
        it = out["iters"].cpu().numpy()
        sel = np.nonzero(it > 0)[0]
        print(f"period {s}: {len(sel)} handed over, max iters {int(it.max())}", flush=True)
        if prev is None:
            continue
        w = out["window"]
        for i in sel:
            keep["xi_init"].append(xi0[i].cpu().numpy())
            for k in ("omega", "xi_ref", "vrp_ref", "A", "b", "nfacets"):
                keep[k].append(w[k][i].cpu().numpy())
            keep["vrp_ws"].append(prev["vrp"][i].cpu().numpy())
            keep["lam_ws"].append(prev["lam"][i].cpu().numpy())
            # the status the warm solve was given (the loop's cold-after-hand-over rule applied)
            keep["prev_status"].append(int((loop.warm_status if loop.cold_after_handover else prev["status"])[i]))
            keep["period"].append(s)
            keep["iters"].append(int(it[i]))
    cap = {k: np.asarray(v) for k, v in keep.items()}
    n = len(cap["period"])
    dev = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).cuda()
    prob = {k: dev(cap[k]) for k in ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b")}
    prob["nfacets"] = dev(cap["nfacets"], torch.int32)
    prm = native.default_params(N)
    prm.max_iter = DL.MAX_ITER
    prm.tol_polish = loop.params.tol_polish
    prm.dt = loop.params.dt
    warm = dict(vrp=dev(cap["vrp_ws"]), lam=dev(cap["lam_ws"]), shift=1, floor=1e-3,
                status=dev(cap["prev_status"], torch.int32))
    ow = h.dcm_mpc_solve(prob, prm, warm=warm)
    cold = dict(warm, status=dev(np.ones(n, np.int32), torch.int32))
    oc = h.dcm_mpc_solve(prob, prm, warm=cold)
    torch.cuda.synchronize()
    iw, ic = ow["iters"].cpu().numpy(), oc["iters"].cpu().numpy()
    sw, sc = ow["status"].cpu().numpy(), oc["status"].cpu().numpy()
    print(f"{n} windows: loop iters == warm re-solve: {int((iw == cap['iters']).sum())}; status warm "
          f"{np.bincount(sw).tolist()} cold {np.bincount(sc).tolist()}")
    print(f"iterations warm mean {iw.mean():.1f} max {iw.max()}, cold mean {ic.mean():.1f} max {ic.max()}; "
          f"warm > cold in {int((iw > ic).sum())}, cold > warm in {int((ic > iw).sum())}")
    for s in sorted(set(cap["period"].tolist())):
        m = cap["period"] == s
        print(f"  period {s}: {int(m.sum())} windows, slowest warm {iw[m].max()} cold {ic[m].max()} "
              f"min(warm, cold) {np.minimum(iw, ic)[m].max()}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "c5_handover_starts.npz"), iters_warm=iw, iters_cold=ic, **cap)


if __name__ == "__main__":
    main()
