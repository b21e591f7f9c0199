"""CPU tests of the floating-base dynamics oracle (oracle/fb_dynamics.py), the checker of the
blf_fbd_* kernels.  The reference's rigid-body terms come from iDynTree,
absent here, and the reference has no test for this class, so parity is UNPINNED;
the oracle is validated by self-consistency at several random states of the synthetic 30-DoF
model (blf/robot.py):
  * M symmetric positive definite, M[0:3, 0:3] = total mass I;
  * 1/2 nu^T M nu equals the kinetic energy summed link by link;
  * nu^T h(g = 0) = 1/2 nu^T (dM/dt) nu  (skew-symmetry of dM/dt - 2C; dM/dt by central differences
    along the motion);
  * nu^T (h - h(g = 0)) = dV/dt = -sum_l m_l g . v_com,l;
  * the equation of motion M nu_dot + h = [0; tau] + sum_c J_c^T w_c holds for the solution."""
import numpy as np
import pytest

import fb_dynamics as F
import oracle as O
from blf import robot

MODEL = robot.humanoid24()
# the same tree with four joints prismatic (URDF "prismatic": the child slides along the axis):
# a leaf (neck), an inner torso joint, a knee and a hip, so every identity below also covers the
# prismatic kinematics, Jacobian columns and bias terms (oracle/fb_dynamics.py)
PRISMATIC = ("neck_pitch", "torso_roll", "l_knee", "r_hip_pitch")
MODEL_P = robot.with_joint_types(MODEL, prismatic=PRISMATIC)
MODELS = {"revolute": MODEL, "prismatic": MODEL_P}


def state_i(st, i):
    return {k: v[i] for k, v in st.items()}


@pytest.mark.parametrize("kind", sorted(MODELS))
@pytest.mark.parametrize("seed", range(3))
def test_mass_matrix_and_energy(seed, kind):
    MODEL = MODELS[kind]
    st = state_i(robot.random_states(MODEL, 1, seed=seed), 0)
    K = F.kinematics(MODEL, st["base_pos"], st["base_rot"], st["joint_pos"], st["base_vel"],
                     st["joint_vel"])
    M, h = F.mass_and_bias(MODEL, K)
    assert np.abs(M - M.T).max() < 1e-13
    assert np.linalg.eigvalsh(M).min() > 0
    np.testing.assert_allclose(M[:3, :3], MODEL["link_mass"].sum() * np.eye(3), atol=1e-12)
    nu = np.concatenate([st["base_vel"], st["joint_vel"]])
    T = 0.0
    for l in range(MODEL["n"] + 1):
        R = K["R"][l]
        c = K["p"][l] + R @ MODEL["link_com"][l]
        vc = K["v"][l] + np.cross(K["w"][l], c - K["p"][l])
        T += 0.5 * MODEL["link_mass"][l] * vc @ vc
        T += 0.5 * K["w"][l] @ (R @ MODEL["link_inertia"][l] @ R.T) @ K["w"][l]
    assert abs(0.5 * nu @ M @ nu - T) < 1e-12 * max(1.0, T)


@pytest.mark.parametrize("kind", sorted(MODELS))
@pytest.mark.parametrize("seed", range(3))
def test_bias_forces_power_identities(seed, kind):
    MODEL = MODELS[kind]
    st = state_i(robot.random_states(MODEL, 1, seed=10 + seed), 0)
    K = F.kinematics(MODEL, st["base_pos"], st["base_rot"], st["joint_pos"], st["base_vel"],
                     st["joint_vel"])
    M, h = F.mass_and_bias(MODEL, K)
    _, h0 = F.mass_and_bias(MODEL, K, gravity=np.zeros(3))
    nu = np.concatenate([st["base_vel"], st["joint_vel"]])
    dt = 1e-6
    w = st["base_vel"][3:]

    def M_at(sign):
        Rn = F.rot_axis(w / np.linalg.norm(w), sign * dt * np.linalg.norm(w)) @ st["base_rot"]
        K2 = F.kinematics(MODEL, st["base_pos"] + sign * dt * st["base_vel"][:3], Rn,
                          st["joint_pos"] + sign * dt * st["joint_vel"], st["base_vel"],
                          st["joint_vel"])
        return F.mass_and_bias(MODEL, K2)[0]

    Mdot = (M_at(1) - M_at(-1)) / (2 * dt)
    assert abs(nu @ h0 - 0.5 * nu @ Mdot @ nu) < 1e-7 * max(1.0, abs(nu @ h0))
    dV = 0.0
    for l in range(MODEL["n"] + 1):
        c = K["p"][l] + K["R"][l] @ MODEL["link_com"][l]
        vc = K["v"][l] + np.cross(K["w"][l], c - K["p"][l])
        dV -= MODEL["link_mass"][l] * F.G @ vc
    assert abs(nu @ (h - h0) - dV) < 1e-10 * max(1.0, abs(dV))


def contact_setup(B, seed=0):
    rng = np.random.default_rng(seed)
    params = np.array([[0.12, 0.09, 3.0e4, 300.0]] * 2)
    null = np.zeros((B, 2, 12))
    null[:, :, :3] = rng.normal(size=(B, 2, 3)) * 0.01
    null[:, :, 3:] = np.eye(3).reshape(-1)
    return np.array([0, 1], dtype=np.int32), params, null


@pytest.mark.parametrize("kind", sorted(MODELS))
def test_equation_of_motion_with_contacts(kind):
    MODEL = MODELS[kind]
    st = robot.random_states(MODEL, 2, seed=4)
    frames, params, null = contact_setup(2)
    for i in range(2):
        ba, ja, dp, dR, dq = F.dynamics(MODEL, st, i, contacts=frames, contact_params=params,
                                        null_poses=null[i])
        s = state_i(st, i)
        K = F.kinematics(MODEL, s["base_pos"], s["base_rot"], s["joint_pos"], s["base_vel"],
                         s["joint_vel"])
        M, h = F.mass_and_bias(MODEL, K)
        rhs = -h.copy()
        rhs[6:] += s["joint_torque"]
        for c, f in enumerate(frames):
            pf, Rf, vel, J = F.frame_state(MODEL, K, f)
            wr = O.contact_eval(params[c], vel, np.concatenate([pf, Rf.reshape(-1)]), null[i][c])[0]
            rhs += J.T @ wr
        acc = np.concatenate([ba, ja])
        np.testing.assert_allclose(M @ acc, rhs, atol=1e-8 * np.abs(rhs).max())
        np.testing.assert_array_equal(dp, s["base_vel"][:3])
        np.testing.assert_array_equal(dq, s["joint_vel"])


@pytest.mark.parametrize("kind", sorted(MODELS))
def test_frame_jacobian_matches_frame_velocity(kind):
    MODEL = MODELS[kind]
    st = state_i(robot.random_states(MODEL, 1, seed=8), 0)
    K = F.kinematics(MODEL, st["base_pos"], st["base_rot"], st["joint_pos"], st["base_vel"],
                     st["joint_vel"])
    nu = np.concatenate([st["base_vel"], st["joint_vel"]])
    for f in range(2):
        _, _, vel, J = F.frame_state(MODEL, K, f)
        np.testing.assert_allclose(J @ nu, vel, atol=1e-13)


# Fixed joints (blf/robot.py reduce_fixed_joints): a leaf (neck_pitch), an inner joint with
# children (torso_roll), a chain of two (the left shoulder roll + yaw), and a joint whose child
# carries a sole frame (l_ankle_roll).
FIXED = ("neck_pitch", "torso_roll", "l_shoulder_roll", "l_shoulder_yaw", "l_ankle_roll")


@pytest.mark.parametrize("seed", range(3))
def test_fixed_joints_reduce_to_the_locked_model(seed):
    """The reduced model's rigid-body terms equal the full model's with the fixed joints held at
    q = 0, q_dot = 0 (their rows and columns removed); the sole frames' poses and Jacobians too."""
    red = robot.reduce_fixed_joints(MODEL, FIXED)
    keep_j = [j for j in range(MODEL["n"]) if MODEL["names"][j + 1] not in FIXED]
    assert red["n"] == MODEL["n"] - len(FIXED) and red["names"][1:] == [MODEL["names"][j + 1] for j in keep_j]
    assert abs(red["link_mass"].sum() - MODEL["link_mass"].sum()) < 1e-12
    st = state_i(robot.random_states(MODEL, 1, seed=30 + seed), 0)
    qf, vf = st["joint_pos"].copy(), st["joint_vel"].copy()
    for name in FIXED:
        j = MODEL["names"].index(name) - 1
        qf[j] = 0.0
        vf[j] = 0.0
    K = F.kinematics(MODEL, st["base_pos"], st["base_rot"], qf, st["base_vel"], vf)
    M, h = F.mass_and_bias(MODEL, K)
    Kr = F.kinematics(red, st["base_pos"], st["base_rot"], qf[keep_j], st["base_vel"], vf[keep_j])
    Mr, hr = F.mass_and_bias(red, Kr)
    rows = list(range(6)) + [6 + j for j in keep_j]
    np.testing.assert_allclose(Mr, M[np.ix_(rows, rows)], rtol=1e-12, atol=1e-12 * np.abs(M).max())
    np.testing.assert_allclose(hr, h[rows], rtol=1e-12, atol=1e-12 * np.abs(h).max())
    for f in range(len(MODEL["frame_link"])):
        pf, Rf, vel, J = F.frame_state(MODEL, K, f)
        pr, Rr, velr, Jr = F.frame_state(red, Kr, f)
        np.testing.assert_allclose(pr, pf, atol=1e-14)
        np.testing.assert_allclose(Rr, Rf, atol=1e-14)
        np.testing.assert_allclose(velr, vel, atol=1e-13)
        np.testing.assert_allclose(Jr, J[:, rows], atol=1e-14)


def test_fixed_joints_argument_errors():
    with pytest.raises(ValueError):
        robot.reduce_fixed_joints(MODEL, [99])
    same = robot.reduce_fixed_joints(MODEL, [])
    for k in ("parent", "joint_origin", "joint_rot", "link_inertia", "frame_pose"):
        np.testing.assert_array_equal(same[k], MODEL[k])


def test_fixed_joints_reject_inconsistent_models():
    """reduce_fixed_joints re-indexes in place, so a non-topological model or one with
    inconsistent array sizes is refused instead of being merged wrong."""
    bad = dict(MODEL, parent=np.array(MODEL["parent"]).copy())
    bad["parent"][3] = 7                          # joint 3 hangs from a later link
    with pytest.raises(ValueError, match="topological"):
        robot.reduce_fixed_joints(bad, FIXED)
    short = dict(MODEL, link_mass=np.asarray(MODEL["link_mass"])[:-1])
    with pytest.raises(ValueError, match="link_mass"):
        robot.reduce_fixed_joints(short, FIXED)


def test_given_wrench_law_is_the_jacobian_transpose_map():
    """A BLF_CONTACT_WRENCH contact (any ContactModel's wrench, FloatingBaseSystemDynamics.cpp:
    198-228): nu_dot(w) - nu_dot(0) = M^-1 J_c^T w, and the continuous model's own wrench given
    this way reproduces the continuous law."""
    st = robot.random_states(MODEL, 2, seed=17)
    frames = np.array([0, 1], dtype=np.int32)
    params = np.array([[0.12, 0.09, 3.0e4, 300.0]] * 2)
    null = np.zeros((2, 12))
    null[:, 3:] = np.eye(3).reshape(-1)
    w = np.array([[10.0, -5.0, 200.0, 1.0, -2.0, 0.5], [-3.0, 4.0, 150.0, 0.2, 0.1, -0.3]])
    kw = dict(contacts=frames, contact_params=params, null_poses=null)
    laws = np.array([F.CONTACT_WRENCH, F.CONTACT_WRENCH])
    a1 = F.dynamics(MODEL, st, 0, laws=laws, wrenches=w, **kw)
    a0 = F.dynamics(MODEL, st, 0, laws=laws, wrenches=np.zeros((2, 6)), **kw)
    s = {k: v[0] for k, v in st.items()}
    K = F.kinematics(MODEL, s["base_pos"], s["base_rot"], s["joint_pos"], s["base_vel"], s["joint_vel"])
    M, _ = F.mass_and_bias(MODEL, K)
    rhs = sum(F.frame_state(MODEL, K, f)[3].T @ w[c] for c, f in enumerate(frames))
    d = np.linalg.solve(M, rhs)
    got = np.concatenate([a1[0] - a0[0], a1[1] - a0[1]])
    np.testing.assert_allclose(got, d, rtol=1e-9, atol=1e-9 * np.abs(d).max())
    cont = F.dynamics(MODEL, st, 0, **kw)
    wc = []
    for c, f in enumerate(frames):
        pf, Rf, vel, _ = F.frame_state(MODEL, K, f)
        wc.append(O.contact_eval(params[c], vel, np.concatenate([pf, Rf.reshape(-1)]), null[c])[0])
    given = F.dynamics(MODEL, st, 0, laws=laws, wrenches=np.array(wc), **kw)
    np.testing.assert_array_equal(given[1], cont[1])
