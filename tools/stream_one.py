"""Run one streaming kernel a few times (for rocprofv3 counter passes):
  python tools/stream_one.py rollout|hull|quintic|contact|fbk|fbk_euler|fbd_euler
fbd_euler: the config-5 dynamics kernel alone, one control period of 16 384 robots
(blf_fbd_euler_integrate_impedance over ClosedLoop's interval: 19 ForwardEuler steps, two
contact feet)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))
from blf import native  # noqa: E402


def main(which):
    h = native.Handle(0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: torch.rand(*s, dtype=torch.float64, device=dev, generator=g)
    if which == "rollout":
        B, N = 262144, 100
        xi0, om, vrp = rnd(B, 2), rnd(B, N) * 4 + 3, rnd(B, N, 2)
        out = torch.empty(B, N + 1, 2, dtype=torch.float64, device=dev)
        fn = lambda: h.dcm_euler_rollout(xi0, om, vrp, 0.02, out=out)
    elif which == "hull":
        P = 2 * 1024 * 1024
        ang = rnd(P, 8) * 6.283
        pts = torch.stack([torch.cos(ang), torch.sin(ang)], dim=-1).contiguous()
        npts = torch.full((P,), 8, dtype=torch.int32, device=dev)
        fn = lambda: h.hull2d_hrep(pts, npts, 8)
    elif which == "quintic":
        S, Q = 1024 * 1024, 32
        kt = torch.cumsum(rnd(S, 3) + 0.1, dim=1).contiguous()
        co = h.quintic_fit(kt, rnd(S, 3, 3, 3))
        tq = (kt[:, :1] + (kt[:, 2:] - kt[:, :1]) * rnd(S, Q)).contiguous()
        fn = lambda: h.quintic_eval(kt, co, tq)
    elif which in ("fbd_euler", "fbd_euler_big"):
        import numpy as np
        from blf import closed_loop as DL
        from blf import robot as R
        B = int(os.environ.get("FBD_BATCH", 16384))
        model = R.humanoid24()
        if which == "fbd_euler_big":   # 4 extra leaf joints on the torso: NV = 34, one system per wavefront
            model = dict(model)
            n0, extra = model["n"], 4
            torso = model["names"].index("torso_pitch")
            model["n"] = n0 + extra
            model["parent"] = np.concatenate([model["parent"], np.full(extra, torso)]).astype(np.int32)
            model["joint_origin"] = np.concatenate([model["joint_origin"], np.tile([[0.0, 0.01, 0.05]], (extra, 1))])
            model["joint_rot"] = np.concatenate([model["joint_rot"], np.tile(np.eye(3), (extra, 1, 1))])
            model["joint_axis"] = np.concatenate([model["joint_axis"], np.tile([[0.0, 0.0, 1.0]], (extra, 1))])
            model["link_mass"] = np.concatenate([model["link_mass"], np.full(extra, 0.3)])
            model["link_com"] = np.concatenate([model["link_com"], np.zeros((extra, 3))])
            model["link_inertia"] = np.concatenate([model["link_inertia"], np.tile(np.eye(3) * 1e-3, (extra, 1, 1))])
            model["names"] = list(model["names"]) + [f"extra{i}" for i in range(extra)]
        st = R.standing_states(model, B, seed=1000)
        law = R.posture_law_arrays(model)
        t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(dev)
        dm = h.fb_model(model)
        state = {k: t(st[k]) for k in native.FB_STATE_KEYS}
        C = len(model["frame_link"])
        contacts = dict(frame=t(np.arange(C), torch.int32),
                        params=t(np.tile(np.asarray(DL.CONTACT_PARAMS, np.float64), (C, 1))),
                        null_pose=t(R.sole_null_poses(model, st)))
        imp = h.joint_impedance(law["kp"], law["kd"])
        q_ref = state["joint_pos"].clone()
        T = DL.period_final_time(0.02, 0.001)
        fn = lambda: h.fbd_euler_integrate_impedance(dm, state, imp, q_ref, 0.0, T, 0.001,
                                                     contacts=contacts)
    elif which in ("fbk", "fbk_euler"):
        B, n = 2 * 1024 * 1024, 24
        R = torch.linalg.qr(torch.randn(B, 3, 3, dtype=torch.float64, device=dev))[0].contiguous()
        tw, sd, pos, q = rnd(B, 6), rnd(B, n), rnd(B, 3), rnd(B, n)
        if which == "fbk":
            fn = lambda: h.fbk_dynamics(0.01, R, tw, sd)
        else:
            fn = lambda: h.fbk_euler_integrate(0.01, pos, R, q, tw, sd, 0.0, 0.01, 0.01)
    else:
        C = 4 * 1024 * 1024
        prm = torch.tensor([0.12, 0.09, 2000.0, 100.0], dtype=torch.float64, device=dev)
        tw, pose, null = rnd(C, 6), rnd(C, 12), rnd(C, 12)
        fn = lambda: h.contact_model_eval(prm, tw, pose, null)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    if os.environ.get("STREAM_TIME"):   # event-timed median of 20 launches
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(40)]
        for i in range(20):
            ev[2 * i].record()
            fn()
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        ms = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(20))
        print(f"{which} lib={os.path.basename(native.LIB_PATH)} median {ms[10]:.4f} ms", flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
