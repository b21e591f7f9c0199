"""GPU parity of the config-5 closed loop (BASELINE.json configs[4]) and
of the configs[3] per-rank shard.

* blf_fb_dcm (state -> centre of mass, DCM), blf_dcm_posture_reference (plan -> joint
  references) and blf_fbd_euler_integrate_impedance against their CPU restatements in
  oracle/closed_loop.py;
* the coupled loop blf.closed_loop.ClosedLoop against oracle/closed_loop.OracleLoop for a few
  control periods: the robot's DCM becomes the plan's xi_init, the plan's first VRP drives the
  robot.  The rigid-body terms agree with the numpy oracle to rounding (1e-9 relative, as in
  test_gpu_fb_dynamics.py; parity vs iDynTree is unpinned), so the loop is
  compared at tolerances, not bit for bit;
* one full-size period of configs[4] (16 384 robots) under size-independent checks;
* a configs[3] shard: 32 768 QPs generated at global offset 7 * 32 768 (rank 7 of 8), a sample
  bit for bit against the oracle.
"""
import numpy as np
import pytest
import torch

import closed_loop as CL
import fb_dynamics as F
from blf import closed_loop as DL
from blf import native, problems as P, robot as R

pytestmark = pytest.mark.gpu
MODEL = R.humanoid24()


def _d(a, dtype=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(a), dtype=dtype).cuda()


def rel_err(a, b):
    return np.abs(a - b).max() / max(1.0, np.abs(b).max())


def test_fb_dcm_vs_oracle(handle):
    B = 64
    st = R.random_states(MODEL, B, seed=4)
    st.pop("joint_torque")
    dm = handle.fb_model(MODEL)
    omega = np.sqrt(9.81 / np.random.default_rng(1).uniform(0.5, 0.6, (B, 7)))
    com, xi = handle.fb_dcm(dm, {k: _d(v) for k, v in st.items()}, omega=_d(omega), column=3)
    torch.cuda.synchronize()
    com_o, xi_o = CL.dcm_from_state(MODEL, st, omega[:, 3])
    assert rel_err(com.cpu().numpy(), com_o) <= 1e-12
    assert rel_err(xi.cpu().numpy(), xi_o) <= 1e-12
    # without omega: the centre of mass alone
    com2, xi2 = handle.fb_dcm(dm, {k: _d(v) for k, v in st.items()})
    assert xi2 is None
    np.testing.assert_array_equal(com2.cpu().numpy(), com.cpu().numpy())


def test_posture_reference_vs_oracle(handle):
    B, N = 96, 50
    rng = np.random.default_rng(2)
    law = R.posture_law_arrays(MODEL)
    com = rng.normal(size=(B, 6)) * 0.05
    vrp = rng.normal(size=(B, N, 2)) * 0.05
    dl = handle.posture_law(law["q_nominal"], law["lean"])
    q_ref = handle.posture_reference(dl, _d(com), _d(vrp))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(q_ref.cpu().numpy(), CL.posture_reference(law, com, vrp))


def test_fbd_euler_impedance_vs_oracle(handle):
    B = 6
    st = R.standing_states(MODEL, B, seed=5)
    law = R.posture_law_arrays(MODEL)
    q_ref = np.random.default_rng(3).normal(size=(B, MODEL["n"])) * 0.02
    null = R.sole_null_poses(MODEL, st)
    cp = np.tile(np.asarray(DL.CONTACT_PARAMS), (2, 1))
    contacts = dict(frame=_d(np.arange(2), torch.int32), params=_d(cp), null_pose=_d(null))
    dev = {k: _d(v) for k, v in st.items()}
    dm = handle.fb_model(MODEL)
    imp = handle.joint_impedance(law["kp"], law["kd"])
    handle.fbd_euler_integrate_impedance(dm, dev, imp, _d(q_ref), 0.0, 0.02, 0.001, contacts=contacts)
    torch.cuda.synchronize()
    for i in range(B):
        ref = CL.euler_integrate_impedance(MODEL, st, i, q_ref[i], law["kp"], law["kd"], 0.0, 0.02,
                                           0.001, contacts=[0, 1], contact_params=cp, null_poses=null[i])
        for k in native.FB_STATE_KEYS:
            assert rel_err(dev[k][i].cpu().numpy(), ref[k]) <= 1e-9, (i, k)


def test_fbd_euler_impedance_zero_gains_is_plain_euler(handle):
    """kp = kd = 0: the impedance sets tau = 0 before every step, the plain integrator with zero
    torques, bit for bit."""
    B = 32
    st = R.standing_states(MODEL, B, seed=6)
    dm = handle.fb_model(MODEL)
    a = {k: _d(v) for k, v in st.items()}
    b = {k: _d(v) for k, v in st.items()}
    n = MODEL["n"]
    imp = handle.joint_impedance(np.zeros(n), np.zeros(n))
    handle.fbd_euler_integrate_impedance(dm, a, imp, _d(np.ones((B, n))), 0.0, 0.01, 0.001)
    handle.fbd_euler_integrate(dm, b, _d(np.zeros((B, n))), 0.0, 0.01, 0.001)
    torch.cuda.synchronize()
    for k in native.FB_STATE_KEYS:
        np.testing.assert_array_equal(a[k].cpu().numpy(), b[k].cpu().numpy())


def test_closed_loop_period_advances_one_knot_of_robot_time(handle):
    """The loop's period integrates exactly one knot dt of robot time (ClosedLoop.T = dt - dT: the
    reference FixedStepIntegrator schedule integrates T + dT, FixedStepIntegrator.tpp:48-64).
    Measured on the device: robots in free fall (no contacts, zero gains, at rest), whose base
    velocity after ForwardEuler is -g times the integrated time, exactly up to rounding."""
    B = 8
    plan, st = _setup(B, 2)
    loop = DL.ClosedLoop(handle, MODEL, plan, st, horizon=100)
    assert abs(sum(loop.steps) - loop.dt) <= 1e-15 and len(loop.steps) == 19
    n = MODEL["n"]
    imp = handle.joint_impedance(np.zeros(n), np.zeros(n))
    g = 9.81

    def fall(t1):
        s = {k: _d(v) for k, v in st.items()}
        s["base_vel"].zero_()
        s["joint_vel"].zero_()
        s["base_pos"][:, 2] += 10.0
        handle.fbd_euler_integrate_impedance(loop.dm, s, imp, s["joint_pos"].clone(), 0.0, t1, loop.dT)
        torch.cuda.synchronize()
        return -s["base_vel"][:, 2].cpu().numpy() / g

    t_loop = fall(loop.T)
    np.testing.assert_allclose(t_loop, loop.dt, rtol=0, atol=1e-12)
    # the reference call integrate(0, dt) itself advances dt + dT (the stale last step)
    np.testing.assert_allclose(fall(loop.dt), loop.dt + loop.dT, rtol=0, atol=1e-12)


def _setup(B, periods, seed=3):
    N = 100
    plan = P.make_batch(B, horizon=N + periods, n_footsteps=8, seed=P.SEED, first_ds=periods + 10)
    st = R.standing_states(MODEL, B, seed=seed)
    return plan, st


def test_closed_loop_vs_oracle(handle):
    """A few coupled control periods: xi_init from the robot, the warm-started plan, the joint
    references from the plan, the impedance-driven dynamics — device vs CPU composition."""
    B, S = 6, 4
    plan, st = _setup(B, S)
    loop = DL.ClosedLoop(handle, MODEL, plan, st)
    ref = CL.OracleLoop(MODEL, plan, st, R.sole_null_poses(MODEL, st), R.posture_law_arrays(MODEL),
                        DL.CONTACT_PARAMS)
    for s in range(S):
        out = loop.period()
        xi_init = loop.xi.cpu().numpy().copy()
        torch.cuda.synchronize()
        o = ref.period()
        np.testing.assert_array_equal(out["status"].cpu().numpy(), o["status"])
        assert (o["status"] == 0).all()
        assert np.abs(xi_init - o["xi_init"]).max() <= 1e-9, s
        assert np.abs(out["vrp"].cpu().numpy() - o["vrp"]).max() <= 1e-8, s
        assert np.abs(out["xi"].cpu().numpy() - o["xi"]).max() <= 1e-8, s
        for k in native.FB_STATE_KEYS:
            assert rel_err(loop.state[k].cpu().numpy(), ref.state[k]) <= 1e-8, (s, k)
    # the plan drives the robot: its joint references move with (r0 - c)
    assert np.abs(loop.q_ref.cpu().numpy()).max() > 0.0


def test_closed_loop_stream_groups_bitwise(handle):
    """The bench's c5 scheduling (bench.py --c5-groups): the robots in three groups, each closed
    loop on its own stream, run the same computation as one loop over all robots, bit for bit
    (the QP, the maps and the dynamics are per robot; the groups only overlap on the device)."""
    B, S = 96, 3
    plan, st = _setup(B, S)
    one = DL.ClosedLoop(handle, MODEL, plan, st)
    groups = DL.split_groups(handle, MODEL, plan, st, 3)
    assert [lp.B for lp in groups] == [32, 32, 32]
    for s in range(S):
        out1 = one.period()
        outs = [lp.period() for lp in groups]
    torch.cuda.synchronize()
    for k in ("xi", "vrp", "status", "iters"):
        np.testing.assert_array_equal(out1[k].cpu().numpy(),
                                      torch.cat([o[k] for o in outs]).cpu().numpy(), err_msg=k)
    for k in native.FB_STATE_KEYS:
        np.testing.assert_array_equal(one.state[k].cpu().numpy(),
                                      torch.cat([lp.state[k] for lp in groups]).cpu().numpy(), err_msg=k)


def test_closed_loop_stage2_list_bitwise(handle):
    """Windows the active-set kernel hands over reach the interior point kernel through the
    stream's pending list (a small grid over the listed problems, csrc/dcm_mpc_ipm.hip).  Pushed
    robots (a lateral base velocity: uncapturable DCM states) make sure some windows take that
    path, period after period; the phase-indexed solve and the expanded-window solve (the per-knot
    input, blf_dcm_phase_expand + blf_dcm_mpc_solve_warm) each list them, and every robot's plan
    and state agree bit for bit.  Every window ends solved (status 0): these QPs are feasible and
    strictly convex, and since round 6 the solver certifies them (round 5
    ended 24 of the 160 windows of a period at MAX_ITER / NUMERICAL; those windows are the fixture
    tests/golden/c5_pushed_windows.npz, certified against dense KKT in tests/test_c5_windows.py)."""
    B, S = 160, 4
    plan, st = _setup(B, S)
    st["base_vel"][::5, 1] += 1.2
    ph = DL.ClosedLoop(handle, MODEL, plan, st)
    ex = DL.ClosedLoop(handle, MODEL, plan, st)
    ex.expand_path = True
    nipm = 0
    for s in range(S):
        out1 = ph.period()
        out2 = ex.period()
        torch.cuda.synchronize()
        nipm += int((out1["iters"] > 0).sum())
        xi0 = out1["xi"][:, 0].cpu().numpy()
        assert np.isfinite(xi0).all(), f"period {s}: non-finite xi_init"
        bad = np.nonzero(out1["status"].cpu().numpy() != 0)[0]
        assert len(bad) == 0, (f"period {s}: unsolved windows", bad.tolist(), out1["status"].cpu().numpy()[bad].tolist())
        for k in ("xi", "vrp", "status", "iters", "polished", "lam"):
            np.testing.assert_array_equal(out1[k].cpu().numpy(), out2[k].cpu().numpy(), err_msg=f"{k} period {s}")
    assert nipm > 0, "no window went to the interior point kernel"
    for k in native.FB_STATE_KEYS:
        np.testing.assert_array_equal(ph.state[k].cpu().numpy(), ex.state[k].cpu().numpy(), err_msg=k)


def test_closed_loop_config5_full_size(handle):
    """configs[4] at its size on one GPU: 16 384 robots, three coupled periods; finite states,
    every plan solved, xi_init = the robot's DCM."""
    B, S = 16384, 3
    plan, st = _setup(B, S)
    loop = DL.ClosedLoop(handle, MODEL, plan, st)
    for s in range(S):
        out = loop.period()
        # every window converges and ends in the certified polish, uncapturable ones included
        # (the c5 bench's "max_iter": 0)
        torch.cuda.synchronize()
        assert int((out["status"] != 0).sum()) == 0, f"period {s}: unsolved windows"
        assert bool((out["polished"] == 1).all()), f"period {s}: unpolished windows"
    for k in native.FB_STATE_KEYS:
        assert torch.isfinite(loop.state[k]).all(), k
    # the last plan started from the robot's DCM (blf_fb_dcm of the state before the period)
    np.testing.assert_array_equal(out["xi"][:, 0].cpu().numpy(), loop.xi.cpu().numpy())
    z = loop.state["base_pos"][:, 2]
    assert float(z.min()) > 0.4 and float(z.max()) < 0.7   # standing, not falling


def test_config3_rank7_shard_bitwise(handle, oracle):
    """configs[3] is 262 144 QPs over 8 GPUs: rank r solves problems [32768 r, 32768 (r + 1)).
    Rank 7's shard on one device, a sample of 256 of its QPs bit for bit against the oracle."""
    B, r = 32768, 7
    prob = P.make_batch(B, horizon=100, n_footsteps=6, seed=P.SEED, start=r * B)
    dev = {k: _d(prob[k]) for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}
    A, b, nf = handle.assemble_constraints(_d(prob["corners"]), _d(prob["ncorners"], torch.int32))
    dev.update(A=A, b=b, nfacets=nf)
    out = handle.dcm_mpc_solve(dev)
    torch.cuda.synchronize()
    assert int((out["status"] != 0).sum()) == 0
    idx = np.random.default_rng(0).choice(B, 256, replace=False)
    host = {k: np.ascontiguousarray(prob[k][idx]) for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}
    for k, v in (("A", A), ("b", b), ("nfacets", nf)):
        host[k] = np.ascontiguousarray(v.cpu().numpy()[idx])
    st, xi, vrp, it = oracle.dcm_mpc_solve_batch(host, threads=8, device_batch=B)   # B-QP launch
    np.testing.assert_array_equal(out["xi"].cpu().numpy()[idx], xi)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy()[idx], vrp)
    np.testing.assert_array_equal(out["iters"].cpu().numpy()[idx], it)
    # the shard is the global problems 7 * 32768 + i: problem 0 of the shard regenerated alone
    one = P.make_batch(1, horizon=100, n_footsteps=6, seed=P.SEED, start=r * B + int(idx[0]))
    np.testing.assert_array_equal(one["xi_init"][0], prob["xi_init"][idx[0]])
