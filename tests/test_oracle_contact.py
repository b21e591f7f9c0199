"""CPU tests of the oracle's restatement of the config-5 rows:
ContinuousContactModel (ContactModels/src/ContinuousContactModel.cpp) and
FloatingBaseSystemKinematics (System/src/FloatingBaseSystemKinematics.cpp).

The reference cannot be built here (Eigen / iDynTree absent), so these restate the reference's own
test, ContactModels/tests/ContinousContactModelTest.cpp, on the oracle: the Monte Carlo integral of
the point forces (tol 1e-2), the regressor identity (tol 1e-7) and the finite-difference consistency
of the wrench rate (tol 1e-4), at the test's configuration (RPY(-0.15, 0.2, 0.1), L = 0.12,
W = 0.09, k = 2000, b = 100).  Eigen's unseeded setRandom twist cannot be reproduced; seeded
uniform(-1, 1) draws stand in for it (parity of the random draw itself is unpinned)."""
import numpy as np
import pytest
from scipy.spatial.transform import Rotation as Rot

import oracle as O

PRM = np.array([0.12, 0.09, 2000.0, 100.0])


def ref_pose():
    # iDynTree Rotation::RPY(r, p, y) = Rz(y) Ry(p) Rx(r) = scipy extrinsic 'xyz'
    R = Rot.from_euler("xyz", [-0.15, 0.2, 0.1]).as_matrix()
    return np.concatenate([[-0.02, 0.01, 0.005], R.reshape(-1)]), R


NULL = np.concatenate([[0.0, 0.0, 0.0], np.eye(3).reshape(-1)])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_contact_wrench_matches_monte_carlo_integral(seed):
    pose, R = ref_pose()
    rng = np.random.default_rng(seed)
    twist = rng.uniform(-1, 1, 6)
    wrench = O.contact_eval(PRM, twist, pose, NULL)[0]
    samples = 10000                                    # ContinousContactModelTest.cpp:70
    xs = rng.uniform(-PRM[0] / 2, PRM[0] / 2, samples)
    ys = rng.uniform(-PRM[1] / 2, PRM[1] / 2, samples)
    F, T = np.zeros(3), np.zeros(3)
    for x, y in zip(xs, ys):
        f, t = O.contact_point(PRM, twist, pose, NULL, x, y)
        F += f
        T += t
    scale = PRM[0] * PRM[1] * abs(R[2, 2]) / samples
    np.testing.assert_allclose(F * scale, wrench[:3], rtol=0, atol=1e-2)
    np.testing.assert_allclose(T * scale, wrench[3:], rtol=0, atol=1e-2)


def test_point_force_is_zero_outside_the_patch():
    pose, _ = ref_pose()
    for x, y in ((0.07, 0.0), (0.0, -0.05), (-0.061, 0.044)):
        f, t = O.contact_point(PRM, np.ones(6), pose, NULL, x, y)
        assert not f.any() and not t.any()


@pytest.mark.parametrize("seed", range(5))
def test_regressor_identity(seed):
    rng = np.random.default_rng(seed)
    pose, _ = ref_pose()
    if seed:
        R = Rot.random(random_state=seed).as_matrix()
        pose = np.concatenate([rng.normal(size=3) * 0.05, R.reshape(-1)])
    twist = rng.uniform(-1, 1, 6)
    wrench, _, _, reg = O.contact_eval(PRM, twist, pose, NULL)
    np.testing.assert_allclose(reg @ PRM[2:], wrench, rtol=0, atol=1e-7)   # tol of the test


@pytest.mark.parametrize("seed", range(3))
def test_wrench_rate_matches_finite_differences(seed):
    # ContinousContactModelTest.cpp "Test contact dynamics": propagate the state by +-h with
    # constant unit spatial acceleration, R(t +- h) = exp(+-skew(w) h) R(t) (mixed representation)
    pose, R = ref_pose()
    twist = np.random.default_rng(seed).uniform(-1, 1, 6)
    acc = np.ones(6)
    h = 1e-6
    _, auto, ctrl, _ = O.contact_eval(PRM, twist, pose, NULL)
    rate = auto + ctrl @ acc

    def at(sign):
        p = pose[:3] + sign * twist[:3] * h
        Rn = Rot.from_rotvec(sign * twist[3:] * h).as_matrix() @ R
        return twist + sign * acc * h, np.concatenate([p, Rn.reshape(-1)])

    vm, pm = at(-1)
    vp, pp = at(1)
    num = (O.contact_eval(PRM, vp, pp, NULL)[0] - O.contact_eval(PRM, vm, pm, NULL)[0]) / (2 * h)
    np.testing.assert_allclose(num, rate, rtol=0, atol=1e-4)


def test_autonomous_dynamics_keeps_the_reference_sign_quirk():
    # the wrench scales by |R22|, the rate terms by R22 (ContinuousContactModel.cpp:127-170):
    # flipping the contact upside down flips the control matrix but not the wrench
    pose, R = ref_pose()
    flip = np.diag([1.0, -1.0, -1.0])
    pose_f = np.concatenate([pose[:3], (R @ flip).reshape(-1)])
    tw = np.array([0.1, -0.2, 0.3, 0.0, 0.0, 0.0])
    w1, _, c1, _ = O.contact_eval(PRM, tw, pose, NULL)
    w2, _, c2, _ = O.contact_eval(PRM, tw, pose_f, NULL)
    assert np.sign(c1[0, 0]) == -np.sign(c2[0, 0])
    np.testing.assert_allclose(w1[:3], w2[:3], rtol=1e-12)


def skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


@pytest.mark.parametrize("seed", range(4))
def test_floating_base_kinematics(seed):
    rng = np.random.default_rng(seed)
    R = Rot.random(random_state=seed).as_matrix()
    twist = rng.normal(size=6)
    sd = rng.normal(size=24)
    dp, dR, dq = O.fbk_dynamics(0.01, R, twist, sd)
    np.testing.assert_array_equal(dp, twist[:3])
    np.testing.assert_array_equal(dq, sd)
    # orthonormal R: the Baumgarte term vanishes, dR = skew(w) R
    np.testing.assert_allclose(dR, skew(twist[3:]) @ R, atol=1e-14)
    # perturbed R: the reference formula evaluated with numpy
    Rp = R + 1e-3 * rng.normal(size=(3, 3))
    _, dRp, _ = O.fbk_dynamics(0.01, Rp, twist, sd)
    ref = -np.cross(Rp.T, twist[3:]).T + 0.01 / 2 * (np.linalg.inv(Rp @ Rp.T) - np.eye(3)) @ Rp
    np.testing.assert_allclose(dRp, ref, atol=1e-13)


def test_floating_base_euler_schedule_and_errors():
    R = Rot.from_euler("z", 0.3).as_matrix()
    twist = np.array([0.1, 0.0, -0.2, 0.0, 0.0, 1.0])
    sd = np.array([1.0, -2.0])
    st, p, Rn, q = O.fbk_euler_integrate(0.01, np.zeros(3), R, np.zeros(2), twist, sd, 0.0,
                                         0.05, 0.01)
    assert st == 0
    # stale-time last step: 5 calls, the positions end at t = 0.06
    np.testing.assert_allclose(p, twist[:3] * 0.06, rtol=1e-12)
    np.testing.assert_allclose(q, sd * 0.06, rtol=1e-12)
    # small-step Euler of dR = skew(w) R tracks exp(skew(w) t) R
    st, _, Rn, _ = O.fbk_euler_integrate(0.01, np.zeros(3), R, np.zeros(2), twist, sd, 0.0,
                                         0.5, 1e-4)
    Rex = Rot.from_rotvec(twist[3:] * (0.5 + 1e-4)).as_matrix() @ R
    np.testing.assert_allclose(Rn, Rex, atol=1e-4)
    assert O.fbk_euler_integrate(0.01, np.zeros(3), R, np.zeros(2), twist, sd, 1.0, 0.0, 0.1)[0] == 4
    assert O.fbk_euler_integrate(0.01, np.zeros(3), R, np.zeros(2), twist, sd, 0.0, 1.0, 0.0)[0] == 4
    assert O.fbk_euler_integrate(0.01, np.zeros(3), R, np.zeros(2), twist, sd, 1.0, 1.0, 0.1)[0] == 5
