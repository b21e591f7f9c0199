"""GPU: a robot loaded from URDF (blf/urdf.py) runs through the floating-base Euler kernel with
foot contacts, against the oracle on the same loaded model (1e-9, as tests/test_gpu_fb_dynamics.py).
The URDF is the synthetic humanoid written out by tests/test_urdf.py with massless sole links on
fixed joints, the torso roll joint prismatic and the neck joint fixed, so the device sees the
model after the loader's merge (23 moving joints, sole frames moved onto the ankle links)."""
import numpy as np
import pytest
import torch

import fb_dynamics as F
from blf import native, robot, urdf
from test_urdf import MODEL, to_urdf

pytestmark = pytest.mark.gpu
TOL = 1e-9


def _d(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def test_urdf_model_euler_with_contacts_vs_oracle(handle):
    m = urdf.load_urdf(to_urdf(MODEL, soles=True, types={"torso_roll": "prismatic", "neck_pitch": "fixed"}),
                       frames=("l_sole", "r_sole"))
    assert m["n"] == MODEL["n"] - 1 and "joint_type" in m
    B = 12
    st = robot.random_states(m, B, seed=11)
    rng = np.random.default_rng(4)
    params = np.array([[0.12, 0.09, 3.0e4, 300.0]] * 2)
    null = np.zeros((B, 2, 12))
    null[:, :, :3] = rng.normal(size=(B, 2, 3)) * 0.01
    null[:, :, 3:] = np.eye(3).reshape(-1)
    frame = np.array([0, 1], dtype=np.int32)
    dev = dict(frame=_d(frame, torch.int32), params=_d(params), null_pose=_d(null))
    dm = handle.fb_model(m)
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    t0, t1, dT = 0.0, 0.003, 0.001
    handle.fbd_euler_integrate(dm, dst, _d(st["joint_torque"]), t0, t1, dT, contacts=dev)
    got = {k: v.cpu().numpy() for k, v in dst.items()}
    for i in (0, 5, 11):
        ref = F.euler_integrate(m, st, i, t0, t1, dT, contacts=frame, contact_params=params,
                                null_poses=null[i])
        for k in native.FB_STATE_KEYS:
            err = np.abs(got[k][i] - ref[k]).max() / max(1.0, np.abs(ref[k]).max())
            assert err < TOL, (k, err)
