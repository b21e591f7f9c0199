"""CPU checks of the config-5 closed loop's restatement (oracle/closed_loop.py) and of the
standing-start inputs (blf/robot.py): the centre-of-mass velocity is the derivative of the
centre of mass along the motion, the impedance integrator with zero gains is the plain
ForwardEuler with zero torques, the posture law's ankle gains put m g / 2 (r0 - c) on each
ankle, and the standing start puts the soles on the ground."""
import numpy as np
import pytest

import closed_loop as CL
import fb_dynamics as F
from blf import robot as R

MODEL = R.humanoid24()


def test_com_velocity_is_the_derivative_of_the_com():
    st = R.random_states(MODEL, 4, seed=9)
    st.pop("joint_torque")
    h = 1e-6
    for i in range(4):
        c0, cd = CL.com_state(MODEL, st, i)
        # move every position along its velocity for h (base rotation by the rotation rate)
        s1 = {k: v.copy() for k, v in st.items()}
        w = st["base_vel"][i, 3:]
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        s1["base_pos"][i] = st["base_pos"][i] + h * st["base_vel"][i, :3]
        s1["base_rot"][i] = (np.eye(3) + h * K) @ st["base_rot"][i]
        s1["joint_pos"][i] = st["joint_pos"][i] + h * st["joint_vel"][i]
        c1, _ = CL.com_state(MODEL, s1, i)
        np.testing.assert_allclose((c1 - c0) / h, cd, atol=1e-5)


def test_impedance_with_zero_gains_is_plain_euler():
    st = R.standing_states(MODEL, 2, seed=1)
    n = MODEL["n"]
    a = CL.euler_integrate_impedance(MODEL, st, 1, np.ones(n), np.zeros(n), np.zeros(n), 0.0, 0.005, 0.001)
    b = F.euler_integrate(MODEL, dict(st, joint_torque=np.zeros((2, n))), 1, 0.0, 0.005, 0.001)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k])


def test_posture_law_ankle_gains():
    law = R.posture_law_arrays(MODEL)
    names = MODEL["names"][1:]
    mg2 = 0.5 * MODEL["link_mass"].sum() * 9.81
    for side in ("l", "r"):
        jp, jr = names.index(f"{side}_ankle_pitch"), names.index(f"{side}_ankle_roll")
        assert np.isclose(law["kp"][jp] * law["lean"][jp, 0], mg2)
        assert np.isclose(law["kp"][jr] * law["lean"][jr, 1], -mg2)
    assert (law["kd"] > 0).all() and (law["kp"] > 0).all()
    com = np.zeros((1, 6))
    vrp = np.zeros((1, 3, 2))
    vrp[0, 0] = (0.01, -0.02)
    q = CL.posture_reference(law, com, vrp)[0]
    assert np.isclose(q[names.index("l_ankle_pitch")], 0.01 * law["lean"][names.index("l_ankle_pitch"), 0])


def test_standing_start_puts_the_soles_on_the_ground():
    st = R.standing_states(MODEL, 3, seed=0, spread=0.0, vel=0.0)
    st["base_rot"][:] = np.eye(3)
    for i in range(3):
        K = F.kinematics(MODEL, st["base_pos"][i], st["base_rot"][i], st["joint_pos"][i],
                         st["base_vel"][i], st["joint_vel"][i])
        for f in range(2):
            pf = F.frame_state(MODEL, K, f)[0]
            assert abs(pf[2]) < 3e-3
    null = R.sole_null_poses(MODEL, st)
    assert null.shape == (3, 2, 12) and (null[:, :, 2] == 0).all()


@pytest.mark.parametrize("prismatic", [(), ("neck_pitch", "torso_roll", "l_knee", "r_hip_pitch")])
def test_c_fbd_restatement_matches_numpy(prismatic):
    """oracle/blf_oracle_fbd.c (the configs[4] CPU baseline's dynamics) against the numpy
    restatement: 20 impedance-driven Euler steps with both soles in contact, to 1e-10; also with
    four joints prismatic (blf_fb_model.joint_type)."""
    import oracle as O
    from blf import closed_loop as DL
    MODEL = R.with_joint_types(globals()["MODEL"], prismatic=prismatic)
    B = 4
    st = R.standing_states(MODEL, B, seed=5)
    st.pop("joint_torque", None)
    law = R.posture_law_arrays(MODEL)
    q_ref = np.random.default_rng(3).normal(size=(B, MODEL["n"])) * 0.02
    null = R.sole_null_poses(MODEL, st)
    cp = np.tile(np.asarray(DL.CONTACT_PARAMS), (2, 1))
    got = O.fbd_euler_impedance_batch(MODEL, st, q_ref, law["kp"], law["kd"], cp, null, 0.0, 0.02,
                                      0.001, threads=2)
    for i in range(B):
        ref = CL.euler_integrate_impedance(MODEL, st, i, q_ref[i], law["kp"], law["kd"], 0.0, 0.02,
                                           0.001, contacts=[0, 1], contact_params=cp,
                                           null_poses=null[i])
        for k in ref:
            if k == "joint_torque":
                continue
            err = np.abs(got[k][i] - ref[k]).max() / max(1.0, np.abs(ref[k]).max())
            assert err <= 1e-10, (i, k, err)


def test_compiled_oracle_loop_matches_numpy_loop():
    """OracleLoop(compiled=True) (C centre of mass and dynamics, the configs[4] CPU baseline) runs
    the same periods as the numpy composition, to 1e-9."""
    from blf import closed_loop as DL
    from blf import problems as P
    N, B = 30, 3
    plan = P.make_batch(B, horizon=N + 2, n_footsteps=4, seed=11, first_ds=12)
    st = R.standing_states(MODEL, B, seed=4)
    args = (MODEL, plan, st, R.sole_null_poses(MODEL, st), R.posture_law_arrays(MODEL),
            DL.CONTACT_PARAMS)
    a = CL.OracleLoop(*args, horizon=N)
    b = CL.OracleLoop(*args, horizon=N, compiled=True, threads=2)
    for _ in range(2):
        ra, rb = a.period(), b.period()
        np.testing.assert_array_equal(ra["status"], rb["status"])
        np.testing.assert_allclose(rb["xi_init"], ra["xi_init"], rtol=0, atol=1e-9)
        for k in a.state:
            np.testing.assert_allclose(b.state[k], a.state[k], rtol=0, atol=1e-9)
