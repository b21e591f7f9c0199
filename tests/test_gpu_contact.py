"""GPU parity of the config-5 kernels through the C ABI:
ContinuousContactModel (blf_contact_model_eval / blf_contact_point_wrench) and
FloatingBaseSystemKinematics (blf_fbk_dynamics / blf_fbk_euler_integrate).  Bit-exact against the
oracle on the same inputs (same expression order, no FMA contraction on either side), plus the
reference test's properties (ContinousContactModelTest.cpp) evaluated on device outputs."""
import numpy as np
import pytest
import torch
from scipy.spatial.transform import Rotation as Rot

from blf import native

pytestmark = pytest.mark.gpu


def _d(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()


def contact_batch(B, seed, flip_some=True):
    rng = np.random.default_rng(seed)
    R = Rot.random(B, random_state=seed).as_matrix()
    if flip_some:   # make some R22 negative: the wrench uses |R22|, the rate terms R22
        R[::3] = R[::3] @ np.diag([1.0, -1.0, -1.0])
    R0 = Rot.random(B, random_state=seed + 1).as_matrix()
    pose = np.concatenate([rng.normal(size=(B, 3)) * 0.02, R.reshape(B, 9)], axis=1)
    null = np.concatenate([rng.normal(size=(B, 3)) * 0.02, R0.reshape(B, 9)], axis=1)
    twist = rng.uniform(-1, 1, (B, 6))
    prm = np.stack([rng.uniform(0.08, 0.2, B), rng.uniform(0.05, 0.12, B),
                    rng.uniform(500, 5000, B), rng.uniform(10, 300, B)], axis=1)
    return prm, twist, pose, null


@pytest.mark.parametrize("B,shared", [(1, False), (257, False), (4096, True)])
def test_contact_model_bitwise_vs_oracle(handle, oracle, B, shared):
    prm, twist, pose, null = contact_batch(B, seed=B)
    if shared:
        prm = prm[0]
    out = handle.contact_model_eval(_d(prm), _d(twist), _d(pose), _d(null))
    ref = oracle.contact_eval_batch(prm, twist, pose, null)
    for name, r in zip(("wrench", "autonomous", "control", "regressor"), ref):
        np.testing.assert_array_equal(out[name].cpu().numpy(), r, err_msg=name)


def test_contact_model_output_subsets(handle, oracle):
    prm, twist, pose, null = contact_batch(64, seed=3)
    full = handle.contact_model_eval(_d(prm), _d(twist), _d(pose), _d(null))
    for subset in (("wrench",), ("regressor",), ("autonomous", "control")):
        part = handle.contact_model_eval(_d(prm), _d(twist), _d(pose), _d(null), outputs=subset)
        assert set(part) == set(subset)
        for k in subset:
            assert torch.equal(part[k], full[k])
    with pytest.raises(native.BlfError) as e:
        handle.contact_model_eval(_d(prm), _d(twist), _d(pose), _d(null), outputs=())
    assert e.value.code == 1


def test_contact_properties_on_device(handle):
    """The reference test's three properties on the device outputs: regressor identity (1e-7),
    FD consistency of the wrench rate (1e-4), Monte Carlo integral of the point forces (1e-2)."""
    R = Rot.from_euler("xyz", [-0.15, 0.2, 0.1]).as_matrix()
    pose = np.concatenate([[-0.02, 0.01, 0.005], R.reshape(-1)])[None]
    null = np.concatenate([[0.0, 0.0, 0.0], np.eye(3).reshape(-1)])[None]
    prm = np.array([0.12, 0.09, 2000.0, 100.0])
    twist = np.random.default_rng(7).uniform(-1, 1, (1, 6))
    out = {k: v.cpu().numpy()[0] for k, v in
           handle.contact_model_eval(_d(prm), _d(twist), _d(pose), _d(null)).items()}
    np.testing.assert_allclose(out["regressor"] @ prm[2:], out["wrench"], atol=1e-7)
    # finite differences (mixed representation propagation, constant unit acceleration)
    h, acc = 1e-6, np.ones(6)
    poses, twists = [], []
    for sgn in (-1, 1):
        Rn = Rot.from_rotvec(sgn * twist[0, 3:] * h).as_matrix() @ R
        poses.append(np.concatenate([pose[0, :3] + sgn * twist[0, :3] * h, Rn.reshape(-1)]))
        twists.append(twist[0] + sgn * acc * h)
    w = handle.contact_model_eval(_d(prm), _d(np.array(twists)), _d(np.array(poses)),
                                  _d(np.repeat(null, 2, 0)), outputs=("wrench",))["wrench"]
    w = w.cpu().numpy()
    np.testing.assert_allclose((w[1] - w[0]) / (2 * h),
                               out["autonomous"] + out["control"] @ acc, atol=1e-4)
    # Monte Carlo over 1e4 device-evaluated points
    rng = np.random.default_rng(42)
    n = 10000
    pts = np.stack([rng.uniform(-0.06, 0.06, n), rng.uniform(-0.045, 0.045, n)], axis=1)[None]
    f, t = handle.contact_point_wrench(_d(prm), _d(twist), _d(pose), _d(null), _d(pts))
    scale = 0.12 * 0.09 * abs(R[2, 2]) / n
    np.testing.assert_allclose(f.sum(1).cpu().numpy()[0] * scale, out["wrench"][:3], atol=1e-2)
    np.testing.assert_allclose(t.sum(1).cpu().numpy()[0] * scale, out["wrench"][3:], atol=1e-2)


def test_contact_point_bitwise_vs_oracle(handle, oracle):
    prm, twist, pose, null = contact_batch(16, seed=11)
    rng = np.random.default_rng(12)
    Q = 33
    pts = np.stack([rng.uniform(-0.11, 0.11, (16, Q)), rng.uniform(-0.07, 0.07, (16, Q))], axis=2)
    f, t = handle.contact_point_wrench(_d(prm), _d(twist), _d(pose), _d(null), _d(pts))
    f, t = f.cpu().numpy(), t.cpu().numpy()
    for q in range(16):
        for j in range(Q):
            fo, to = oracle.contact_point(prm[q], twist[q], pose[q], null[q], *pts[q, j])
            np.testing.assert_array_equal(f[q, j], fo)
            np.testing.assert_array_equal(t[q, j], to)


def fbk_batch(B, n, seed):
    rng = np.random.default_rng(seed)
    R = Rot.random(B, random_state=seed).as_matrix() + 1e-3 * rng.normal(size=(B, 3, 3))
    return (rng.normal(size=(B, 3)), R, rng.normal(size=(B, n)), rng.normal(size=(B, 6)),
            rng.normal(size=(B, n)))


@pytest.mark.parametrize("B,n", [(1, 0), (100, 24), (16384, 24)])
def test_fbk_dynamics_bitwise_vs_oracle(handle, oracle, B, n):
    pos, R, q, twist, sd = fbk_batch(B, n, seed=n + B)
    dp, dR, dq = handle.fbk_dynamics(0.01, _d(R), _d(twist), _d(sd))
    dp, dR, dq = dp.cpu().numpy(), dR.cpu().numpy(), dq.cpu().numpy()
    for i in range(0, B, max(1, B // 64)):
        rp, rR, rq = oracle.fbk_dynamics(0.01, R[i], twist[i], sd[i])
        np.testing.assert_array_equal(dp[i], rp)
        np.testing.assert_array_equal(dR[i], rR)
        np.testing.assert_array_equal(dq[i], rq)


@pytest.mark.parametrize("t0,t1,dT", [(0.0, 0.05, 0.01), (1.0, 1.04, 0.01), (0.0, 0.001, 0.01),
                                      (0.0, 0.3, 0.001)])
def test_fbk_euler_bitwise_vs_oracle(handle, oracle, t0, t1, dT):
    B, n = 130, 24
    pos, R, q, twist, sd = fbk_batch(B, n, seed=5)
    dpos, dR, dq = _d(pos), _d(R), _d(q)
    handle.fbk_euler_integrate(0.01, dpos, dR, dq, _d(twist), _d(sd), t0, t1, dT)
    for i in (0, 1, 63, 64, 129):
        st, p, Rn, qn = oracle.fbk_euler_integrate(0.01, pos[i], R[i], q[i], twist[i], sd[i], t0,
                                                   t1, dT)
        assert st == 0
        np.testing.assert_array_equal(dpos.cpu().numpy()[i], p)
        np.testing.assert_array_equal(dR.cpu().numpy()[i], Rn)
        np.testing.assert_array_equal(dq.cpu().numpy()[i], qn)


def test_fbk_errors(handle):
    pos, R, q, twist, sd = fbk_batch(4, 3, seed=1)
    args = [0.01, _d(pos), _d(R), _d(q), _d(twist), _d(sd)]
    for (t0, t1, dT), code in (((1.0, 0.0, 0.1), 4), ((0.0, 1.0, 0.0), 4), ((1.0, 1.0, 0.1), 5)):
        with pytest.raises(native.BlfError) as e:
            handle.fbk_euler_integrate(*args, t0, t1, dT)
        assert e.value.code == code
    with pytest.raises(native.BlfError) as e:
        handle.fbk_dynamics(0.01, _d(R), _d(twist), _d(np.zeros((4, 65))))
    assert e.value.code == 1
