"""GPU parity of the floating-base dynamics kernels (blf_fbd_dynamics / blf_fbd_euler_integrate,
SURVEY.md 8(a) row 6) against the numpy restatement oracle/fb_dynamics.py on the synthetic
30-DoF model (blf/robot.py).  fp64 throughout; the two sides sum in different orders (LAPACK
Cholesky vs the kernel's right-looking one), so the comparison is at a relative tolerance of
1e-9 on the accelerations (north_star: fp64 error < 1e-9), exact on the kinematic part that does
not go through the mass matrix."""
import numpy as np
import pytest
import torch

import fb_dynamics as F
from blf import native, robot

pytestmark = pytest.mark.gpu
MODEL = robot.humanoid24()
TOL = 1e-9


def _d(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def contacts_for(B, seed=0):
    rng = np.random.default_rng(seed)
    params = np.array([[0.12, 0.09, 3.0e4, 300.0]] * 2)
    null = np.zeros((B, 2, 12))
    null[:, :, :3] = rng.normal(size=(B, 2, 3)) * 0.01
    null[:, :, 3:] = np.eye(3).reshape(-1)
    host = dict(frame=np.array([0, 1], dtype=np.int32), params=params, null_pose=null)
    dev = dict(frame=_d(host["frame"], torch.int32), params=_d(params), null_pose=_d(null))
    return host, dev


def rel_err(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


@pytest.mark.parametrize("with_contacts", [False, True])
def test_fbd_dynamics_vs_oracle(handle, with_contacts):
    B = 96
    st = robot.random_states(MODEL, B, seed=21)
    dm = handle.fb_model(MODEL)
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    host, dev = contacts_for(B) if with_contacts else (None, None)
    out = handle.fbd_dynamics(dm, dst, _d(st["joint_torque"]), contacts=dev)
    out = {k: v.cpu().numpy() for k, v in out.items()}
    for i in range(0, B, 7):
        kw = {}
        if with_contacts:
            kw = dict(contacts=host["frame"], contact_params=host["params"],
                      null_poses=host["null_pose"][i])
        ba, ja, dp, dR, dq = F.dynamics(MODEL, st, i, **kw)
        assert rel_err(out["base_vel"][i], ba) < TOL
        assert rel_err(out["joint_vel"][i], ja) < TOL
        np.testing.assert_array_equal(out["base_pos"][i], dp)
        np.testing.assert_allclose(out["base_rot"][i], dR, atol=1e-15)
        np.testing.assert_array_equal(out["joint_pos"][i], dq)


def test_fbd_mass_regularization(handle):
    B = 8
    st = robot.random_states(MODEL, B, seed=3)
    dm = handle.fb_model(MODEL)
    reg = 0.05 * np.eye(30)
    out = handle.fbd_dynamics(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS},
                              _d(st["joint_torque"]), mass_reg=_d(reg))
    ja = out["joint_vel"].cpu().numpy()
    for i in range(B):
        ref = F.dynamics(MODEL, st, i, reg=reg)[1]
        assert rel_err(ja[i], ref) < TOL


@pytest.mark.parametrize("t0,t1,dT", [(0.0, 0.004, 0.001), (0.0, 0.0025, 0.001)])
def test_fbd_euler_vs_oracle(handle, t0, t1, dT):
    B = 16
    st = robot.random_states(MODEL, B, seed=5)
    host, dev = contacts_for(B, seed=1)
    dm = handle.fb_model(MODEL)
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    handle.fbd_euler_integrate(dm, dst, _d(st["joint_torque"]), t0, t1, dT, contacts=dev)
    got = {k: v.cpu().numpy() for k, v in dst.items()}
    for i in (0, 5, 15):
        ref = F.euler_integrate(MODEL, st, i, t0, t1, dT, contacts=host["frame"],
                                contact_params=host["params"], null_poses=host["null_pose"][i])
        for k in native.FB_STATE_KEYS:
            assert rel_err(got[k][i], ref[k]) < TOL, k


def test_fbd_config5_batch_runs(handle):
    """BASELINE configs[4] size: 16384 systems of the 30-DoF model with two foot contacts."""
    B = 16384
    st = robot.random_states(MODEL, B, seed=9)
    host, dev = contacts_for(B, seed=2)
    dm = handle.fb_model(MODEL)
    out = handle.fbd_dynamics(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS},
                              _d(st["joint_torque"]), contacts=dev)
    acc = out["joint_vel"].cpu().numpy()
    assert np.isfinite(acc).all()
    i = B - 1
    ref = F.dynamics(MODEL, st, i, contacts=host["frame"], contact_params=host["params"],
                     null_poses=host["null_pose"][i])[1]
    assert rel_err(acc[i], ref) < TOL


def test_fbd_errors(handle):
    st = robot.random_states(MODEL, 2, seed=1)
    dm = handle.fb_model(MODEL)
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    tau = _d(st["joint_torque"])
    for (t0, t1, dT), code in (((1.0, 0.0, 0.1), 4), ((0.0, 1.0, -1.0), 4), ((0.5, 0.5, 0.1), 5)):
        with pytest.raises(native.BlfError) as e:
            handle.fbd_euler_integrate(dm, dst, tau, t0, t1, dT)
        assert e.value.code == code


@pytest.mark.parametrize("B", [1, 3, 5])
def test_fbd_two_systems_per_wavefront_odd_batches(handle, B):
    """30-DoF systems run two per wavefront (one per half): odd batches leave the last wavefront
    half empty; it must compute nothing visible (a sentinel row past the batch stays untouched)."""
    st = robot.random_states(MODEL, B + 1, seed=40 + B)
    host, dev = contacts_for(B + 1, seed=3)
    dm = handle.fb_model(MODEL)
    full = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    view = {k: v[:B] for k, v in full.items()}
    sentinel = {k: v[B].clone() for k, v in full.items()}
    cdev = dict(dev, null_pose=dev["null_pose"][:B])
    out = handle.fbd_dynamics(dm, view, _d(st["joint_torque"][:B]), contacts=cdev)
    handle.fbd_euler_integrate(dm, view, _d(st["joint_torque"][:B]), 0.0, 0.003, 0.001, contacts=cdev)
    torch.cuda.synchronize()
    for k in native.FB_STATE_KEYS:
        assert torch.equal(full[k][B], sentinel[k]), k
    acc = out["joint_vel"].cpu().numpy()
    got = {k: v.cpu().numpy() for k, v in view.items()}
    for i in range(B):
        kw = dict(contacts=host["frame"], contact_params=host["params"], null_poses=host["null_pose"][i])
        assert rel_err(acc[i], F.dynamics(MODEL, st, i, **kw)[1]) < TOL
        ref = F.euler_integrate(MODEL, st, i, 0.0, 0.003, 0.001, **kw)
        for k in native.FB_STATE_KEYS:
            assert rel_err(got[k][i], ref[k]) < TOL, (i, k)


def test_fbd_fixed_joints_on_device_match_the_locked_full_model(handle):
    """A model with fixed joints (blf/robot.py reduce_fixed_joints, the DoF-less joints iDynTree
    loads from a URDF) on the device, against the full model with those joints held at q = 0,
    q_dot = 0 on the oracle: the full M and h (and contact Jacobians) with the fixed rows and
    columns removed, then the same LLT solve.  Sole frames sit on a merged link (l_ankle_roll)."""
    import oracle as O
    fixed = ("neck_pitch", "torso_roll", "l_shoulder_roll", "l_shoulder_yaw", "l_ankle_roll")
    red = robot.reduce_fixed_joints(MODEL, fixed)
    keep = [j for j in range(MODEL["n"]) if MODEL["names"][j + 1] not in fixed]
    rows = list(range(6)) + [6 + j for j in keep]
    B = 48
    full = robot.random_states(MODEL, B, seed=77)
    st = {k: (v[:, keep] if k in ("joint_pos", "joint_vel", "joint_torque") else v) for k, v in full.items()}
    host, dev = contacts_for(B, seed=3)
    dm = handle.fb_model(red)
    out = handle.fbd_dynamics(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS}, _d(st["joint_torque"]),
                              contacts=dev)
    out = {k: v.cpu().numpy() for k, v in out.items()}
    for i in range(0, B, 5):
        q = np.zeros(MODEL["n"]); qd = np.zeros(MODEL["n"]); tau = np.zeros(MODEL["n"])
        q[keep], qd[keep], tau[keep] = st["joint_pos"][i], st["joint_vel"][i], st["joint_torque"][i]
        K = F.kinematics(MODEL, full["base_pos"][i], full["base_rot"][i], q, full["base_vel"][i], qd)
        M, h = F.mass_and_bias(MODEL, K)
        known = -h
        for c, f in enumerate(host["frame"]):
            pf, Rf, vel, J = F.frame_state(MODEL, K, f)
            wrench = O.contact_eval(host["params"][c], vel, np.concatenate([pf, Rf.reshape(-1)]),
                                    host["null_pose"][i][c])[0]
            known = known + J.T @ wrench
        known[6:] += tau
        acc = np.linalg.solve(M[np.ix_(rows, rows)], known[rows])
        assert rel_err(out["base_vel"][i], acc[:6]) < TOL
        assert rel_err(out["joint_vel"][i], acc[6:]) < TOL


PRISMATIC = ("neck_pitch", "torso_roll", "l_knee", "r_hip_pitch")


@pytest.mark.parametrize("HWkind", ["two_per_wave", "one_per_wave"])
def test_fbd_prismatic_joints_vs_oracle(handle, HWkind):
    """Prismatic joints (blf_fb_model.joint_type, URDF "prismatic") on the device against the numpy
    oracle, whose prismatic kinematics / Jacobian columns the CPU identities of
    tests/test_fb_dynamics.py pin (energy, power, frame velocity): dynamics with both sole
    contacts, then a short Euler integration.  "one_per_wave": the same model with enough extra
    leaf joints to exceed 26 DoF (one system per wavefront)."""
    model = robot.with_joint_types(MODEL, prismatic=PRISMATIC)
    if HWkind == "one_per_wave":   # NV = n + 6 > 32: fbd kernels with one system per wavefront
        model = dict(model)
        extra = 4
        n0 = model["n"]
        model["n"] = n0 + extra
        torso = model["names"].index("torso_pitch")   # the extra leaves hang off the torso link
        model["parent"] = np.concatenate([model["parent"], np.full(extra, torso)]).astype(np.int32)
        model["joint_origin"] = np.concatenate([model["joint_origin"], np.tile([[0.0, 0.01, 0.05]], (extra, 1))])
        model["joint_rot"] = np.concatenate([model["joint_rot"], np.tile(np.eye(3), (extra, 1, 1))])
        model["joint_axis"] = np.concatenate([model["joint_axis"], np.tile([[0.0, 0.0, 1.0]], (extra, 1))])
        model["link_mass"] = np.concatenate([model["link_mass"], np.full(extra, 0.3)])
        model["link_com"] = np.concatenate([model["link_com"], np.zeros((extra, 3))])
        model["link_inertia"] = np.concatenate([model["link_inertia"], np.tile(np.eye(3) * 1e-3, (extra, 1, 1))])
        model["joint_type"] = np.concatenate([model["joint_type"], np.array([1, 0, 1, 0], dtype=np.int32)])
        model["names"] = list(model["names"]) + [f"extra{i}" for i in range(extra)]
    B = 40
    st = robot.random_states(model, B, seed=9)
    host, dev = contacts_for(B, seed=2)
    dm = handle.fb_model(model)
    out = handle.fbd_dynamics(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS}, _d(st["joint_torque"]),
                              contacts=dev)
    out = {k: v.cpu().numpy() for k, v in out.items()}
    for i in range(0, B, 3):
        ba, ja, dp, dR, dq = F.dynamics(model, st, i, contacts=host["frame"], contact_params=host["params"],
                                        null_poses=host["null_pose"][i])
        assert rel_err(out["base_vel"][i], ba) < TOL
        assert rel_err(out["joint_vel"][i], ja) < TOL
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    handle.fbd_euler_integrate(dm, dst, _d(st["joint_torque"]), 0.0, 0.0035, 0.001, contacts=dev)
    got = {k: v.cpu().numpy() for k, v in dst.items()}
    for i in (0, 7, B - 1):
        ref = F.euler_integrate(model, st, i, 0.0, 0.0035, 0.001, contacts=host["frame"],
                                contact_params=host["params"], null_poses=host["null_pose"][i])
        for k in native.FB_STATE_KEYS:
            assert rel_err(got[k][i], ref[k]) < TOL, k


def test_fbd_unknown_joint_type(handle):
    """An unknown blf_fb_model.joint_type is never taken as revolute.  The Python wrapper refuses it
    (ValueError); through the C ABI (the device array overwritten in place) every output of every
    robot is NaN, in the dynamics and in the Euler integration."""
    model = robot.with_joint_types(MODEL, prismatic=PRISMATIC)
    bad = dict(model)
    bad["joint_type"] = np.array(model["joint_type"]).copy()
    bad["joint_type"][3] = 7
    with pytest.raises(ValueError):
        handle.fb_model(bad)
    B = 8
    st = robot.random_states(model, B, seed=19)
    host, dev = contacts_for(B, seed=4)
    dm = handle.fb_model(model)
    dm.t["joint_type"][3] = 7   # what a C caller could pass
    out = handle.fbd_dynamics(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS}, _d(st["joint_torque"]),
                              contacts=dev)
    for k in ("base_vel", "joint_vel"):   # the accelerations (the rest of the derivative is the state's)
        assert torch.isnan(out[k]).all(), k
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    handle.fbd_euler_integrate(dm, dst, _d(st["joint_torque"]), 0.0, 0.002, 0.001, contacts=dev)
    for k in ("base_vel", "joint_vel", "base_pos", "base_rot"):
        assert torch.isnan(dst[k]).all(), k


# ---- contact laws (blf_fb_contacts.law): any ContactModel through its wrench --------------------
def test_fb_frame_state_vs_oracle(handle):
    """blf_fb_frame_state: world transform and mixed twist of the sole frames, the state the
    reference hands each contact model (FloatingBaseSystemDynamics.cpp:225-226)."""
    B = 24
    st = robot.random_states(MODEL, B, seed=31)
    dm = handle.fb_model(MODEL)
    frames = np.array([1, 0, 1], dtype=np.int32)
    pose, twist = handle.fb_frame_state(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS},
                                        _d(frames, torch.int32))
    pose, twist = pose.cpu().numpy(), twist.cpu().numpy()
    for i in range(0, B, 5):
        K = F.kinematics(MODEL, st["base_pos"][i], st["base_rot"][i], st["joint_pos"][i],
                         st["base_vel"][i], st["joint_vel"][i])
        for c, f in enumerate(frames):
            pf, Rf, vel, _ = F.frame_state(MODEL, K, f)
            np.testing.assert_allclose(pose[i, c], np.concatenate([pf, Rf.reshape(-1)]), rtol=0, atol=1e-12)
            np.testing.assert_allclose(twist[i, c], vel, rtol=0, atol=1e-12 * max(1.0, np.abs(vel).max()))


def _mixed_contacts(B, seed):
    """Contact 0 a ContinuousContactModel, contact 1 BLF_CONTACT_WRENCH with a random wrench."""
    host, dev = contacts_for(B, seed=seed)
    rng = np.random.default_rng(seed + 100)
    wrench = rng.normal(size=(B, 2, 6)) * np.array([40.0, 40.0, 300.0, 5.0, 5.0, 2.0])
    law = np.array([native.CONTACT_CONTINUOUS, native.CONTACT_WRENCH], dtype=np.int32)
    host = dict(host, law=law, wrench=wrench)
    dev = dict(dev, law=_d(law, torch.int32), wrench=_d(wrench))
    return host, dev


@pytest.mark.parametrize("HWkind", ["two_per_wave", "one_per_wave"])
def test_fbd_mixed_contact_laws_vs_oracle(handle, HWkind):
    """A continuous contact and a given-wrench contact (any other ContactModel, evaluated by the
    caller) in one launch: dynamics and a short Euler integration against the numpy oracle."""
    model = MODEL if HWkind == "two_per_wave" else robot.with_joint_types(MODEL, prismatic=PRISMATIC)
    if HWkind == "one_per_wave":   # NV > 32: one system per wavefront
        model = dict(model)
        extra = 4
        torso = model["names"].index("torso_pitch")
        model["n"] = model["n"] + extra
        model["parent"] = np.concatenate([model["parent"], np.full(extra, torso)]).astype(np.int32)
        model["joint_origin"] = np.concatenate([model["joint_origin"], np.tile([[0.0, 0.01, 0.05]], (extra, 1))])
        model["joint_rot"] = np.concatenate([model["joint_rot"], np.tile(np.eye(3), (extra, 1, 1))])
        model["joint_axis"] = np.concatenate([model["joint_axis"], np.tile([[0.0, 0.0, 1.0]], (extra, 1))])
        model["link_mass"] = np.concatenate([model["link_mass"], np.full(extra, 0.3)])
        model["link_com"] = np.concatenate([model["link_com"], np.zeros((extra, 3))])
        model["link_inertia"] = np.concatenate([model["link_inertia"], np.tile(np.eye(3) * 1e-3, (extra, 1, 1))])
        model["joint_type"] = np.concatenate([model["joint_type"], np.zeros(extra, dtype=np.int32)])
        model["names"] = list(model["names"]) + [f"extra{i}" for i in range(extra)]
    B = 21
    st = robot.random_states(model, B, seed=12)
    host, dev = _mixed_contacts(B, seed=4)
    dm = handle.fb_model(model)
    out = handle.fbd_dynamics(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS}, _d(st["joint_torque"]),
                              contacts=dev)
    out = {k: v.cpu().numpy() for k, v in out.items()}
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    handle.fbd_euler_integrate(dm, dst, _d(st["joint_torque"]), 0.0, 0.003, 0.001, contacts=dev)
    got = {k: v.cpu().numpy() for k, v in dst.items()}
    for i in range(0, B, 4):
        kw = dict(contacts=host["frame"], contact_params=host["params"], null_poses=host["null_pose"][i],
                  laws=host["law"], wrenches=host["wrench"][i])
        ba, ja, dp, dR, dq = F.dynamics(model, st, i, **kw)
        assert rel_err(out["base_vel"][i], ba) < TOL
        assert rel_err(out["joint_vel"][i], ja) < TOL
        # the given wrench matters: the continuous law in its place gives other accelerations
        alt = F.dynamics(model, st, i, **dict(kw, laws=None))[1]
        assert rel_err(alt, ja) > 1e-6
        ref = F.euler_integrate(model, st, i, 0.0, 0.003, 0.001, **kw)
        for k in native.FB_STATE_KEYS:
            assert rel_err(got[k][i], ref[k]) < TOL, (i, k)


def test_fbd_given_wrench_of_the_continuous_model_equals_the_continuous_law(handle):
    """The C++ adapter's path for a ContactModel the kernel does not know: frame state on the
    device, the model's wrench at that state, BLF_CONTACT_WRENCH.  With the ContinuousContactModel
    itself evaluated that way (blf_contact_model_eval) the dynamics equal the in-kernel law."""
    B = 32
    st = robot.random_states(MODEL, B, seed=8)
    host, dev = contacts_for(B, seed=6)
    dm = handle.fb_model(MODEL)
    dst = {k: _d(st[k]) for k in native.FB_STATE_KEYS}
    tau = _d(st["joint_torque"])
    pose, twist = handle.fb_frame_state(dm, dst, dev["frame"])
    C = 2
    prm = dev["params"].repeat(B, 1).contiguous()
    w = handle.contact_model_eval(prm, twist.reshape(B * C, 6).contiguous(), pose.reshape(B * C, 12).contiguous(),
                                  dev["null_pose"].reshape(B * C, 12).contiguous(), outputs=("wrench",))["wrench"]
    law = _d(np.array([native.CONTACT_WRENCH] * C, dtype=np.int32), torch.int32)
    given = dict(dev, law=law, wrench=w.reshape(B, C, 6).contiguous())
    a = handle.fbd_dynamics(dm, dst, tau, contacts=dev)
    b = handle.fbd_dynamics(dm, dst, tau, contacts=given)
    for k in ("base_vel", "joint_vel"):
        x, y = a[k].cpu().numpy(), b[k].cpu().numpy()
        assert np.abs(x - y).max() <= 1e-12 * max(1.0, np.abs(x).max()), k


def test_fbd_contact_law_without_wrench_is_refused(handle):
    B = 2
    st = robot.random_states(MODEL, B, seed=1)
    host, dev = contacts_for(B)
    dm = handle.fb_model(MODEL)
    bad = dict(dev, law=_d(np.array([0, 1], dtype=np.int32), torch.int32), wrench=None)
    with pytest.raises(native.BlfError) as e:
        handle.fbd_dynamics(dm, {k: _d(st[k]) for k in native.FB_STATE_KEYS}, _d(st["joint_torque"]),
                            contacts=bad)
    assert e.value.code == 1


def test_fb_frame_state_argument_errors(handle):
    """blf_fb_frame_state refuses null frames / outputs and negative sizes with
    BLF_ERR_INVALID_ARGUMENT (no device access)."""
    import ctypes
    B = 2
    st = robot.random_states(MODEL, B, seed=1)
    dm = handle.fb_model(MODEL)
    fs = handle._fb_state({k: _d(st[k]) for k in native.FB_STATE_KEYS}, B, MODEL["n"])
    out = _d(np.zeros((B, 1, 12)))
    L = native.lib()
    frames = _d(np.array([0], dtype=np.int32), torch.int32)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    for args in ((1, None, B, vp(out), None), (1, vp(frames), B, None, None), (-1, vp(frames), B, vp(out), None),
                 (1, vp(frames), -1, vp(out), None)):
        rc = L.blf_fb_frame_state(handle._h, ctypes.byref(dm.c), ctypes.byref(fs), args[0], args[1], args[2],
                                  args[3], args[4], None)
        assert rc == 1, args
