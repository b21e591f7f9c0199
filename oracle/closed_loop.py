"""TEST INFRASTRUCTURE ONLY — the CPU composition of the config-5 closed loop (DESIGN.md section
11), the checker of blf/closed_loop.py and of the blf_fb_dcm / blf_dcm_posture_torque kernels
(tests/ and bench.py's cpu_baseline only).

One control period, as blf.closed_loop.ClosedLoop.period() runs it on the device:
  1. centre of mass c, cdot from the floating-base state (forward kinematics of
     oracle/fb_dynamics.py), xi = c_xy + cdot_xy / omega_0;
  2. the plan window moved one knot: orc_dcm_phase_expand over the oracle hulls of the phases,
     solved warm from the previous period (orc_dcm_mpc_solve_warm, shift 1);
  3. q_ref = q_nom + lean (r0 - c_xy) with r0 the plan's first VRP;
  4. ForwardEuler<FloatingBaseDynamicalSystem>::integrate(0, dt - dT) of every robot (dt of robot
     time: the reference schedule integrates T + dT) with the control
     input tau = kp (q_ref - q) - kd qdot set before every step (FixedStepIntegrator.tpp:21-72,
     ForwardEuler.tpp:18-49 over FloatingBaseSystemDynamics.cpp:102-251, contacts
     ContinuousContactModel.cpp:79-108, through fb_dynamics.dynamics).
The reference has no closed-loop driver of its own; steps 1 and 3 are this build's maps (parity
of the rigid-body terms against iDynTree is unpinned).
"""
import numpy as np

import fb_dynamics as F
import oracle as O


def com_state(model, st, i):
    """(c, cdot) of system i: sum_l m_l (p_l + R_l com_l) / m, sum_l m_l (v_l + w_l x R_l com_l) / m."""
    K = F.kinematics(model, st["base_pos"][i], st["base_rot"][i], st["joint_pos"][i],
                     st["base_vel"][i], st["joint_vel"][i])
    m = model["link_mass"]
    rc = np.einsum("lab,lb->la", K["R"], model["link_com"])
    c = (m[:, None] * (K["p"] + rc)).sum(0) / m.sum()
    cd = (m[:, None] * (K["v"] + np.cross(K["w"], rc))).sum(0) / m.sum()
    return c, cd


def dcm_from_state(model, st, omega0):
    """com [B,6] and xi [B,2] = c_xy + cdot_xy / omega0 (the blf_fb_dcm map)."""
    B = st["base_pos"].shape[0]
    com = np.zeros((B, 6))
    for i in range(B):
        c, cd = com_state(model, st, i)
        com[i, :3], com[i, 3:] = c, cd
    xi = com[:, :2] + com[:, 3:5] / omega0[:, None]
    return com, xi


def posture_reference(law, com, vrp):
    """q_ref = q_nom + lean_0 (r0_x - c_x) + lean_1 (r0_y - c_y) (the blf_dcm_posture_reference
    map; same operation order)."""
    ex = (vrp[:, 0, 0] - com[:, 0])[:, None]
    ey = (vrp[:, 0, 1] - com[:, 1])[:, None]
    return (law["q_nominal"][None, :] + law["lean"][None, :, 0] * ex) + law["lean"][None, :, 1] * ey


def euler_integrate_impedance(model, st, i, q_ref, kp, kd, t0, t1, dT, **kw):
    """ForwardEuler<FloatingBaseDynamicalSystem>::integrate(t0, t1) of system i with the control
    input set before every step to tau = kp (q_ref - q) - kd qdot (the FixedStepIntegrator
    schedule of fb_dynamics.euler_integrate; blf_fbd_euler_integrate_impedance)."""
    s = {k: np.array(v[i], dtype=np.float64) for k, v in st.items()}
    iters = int(np.ceil((t1 - t0) / dT))
    steps = [dT] * (iters - 1)
    cur = t0 + dT * (iters - 2) if iters >= 2 else t0
    steps.append(t1 - cur)
    for h in steps:
        tau = kp * (q_ref - s["joint_pos"]) - kd * s["joint_vel"]
        one = {k: v[None] for k, v in s.items()}
        one["joint_torque"] = tau[None]
        ba, ja, dp, dR, dq = F.dynamics(model, one, 0, **kw)
        s["base_pos"] = s["base_pos"] + dp * h
        s["base_rot"] = s["base_rot"] + dR * h
        s["joint_pos"] = s["joint_pos"] + dq * h
        s["base_vel"] = s["base_vel"] + ba * h
        s["joint_vel"] = s["joint_vel"] + ja * h
    return s


def phase_table(plan, max_facets=8):
    """The plan's phase table with the oracle's support-polygon H-reps (orc_hull2d_hrep)."""
    B, P = plan["phase_begin"].shape
    A = np.zeros((B, P, max_facets, 2))
    b = np.zeros((B, P, max_facets))
    nf = np.zeros((B, P), dtype=np.int32)
    for q in range(B):
        for p in range(P):
            A[q, p], b[q, p], nf[q, p] = O.hull2d_hrep(
                plan["phase_corners"][q, p, :plan["phase_ncorners"][q, p]], max_facets)
    return dict(nphases=plan["nphases"], phase_begin=plan["phase_begin"], phase_end=plan["phase_end"],
                phase_A=A, phase_b=b, phase_nf=nf, phase_ref=plan["phase_ref"])


class OracleLoop:
    """blf.closed_loop.ClosedLoop restated on the CPU (same inputs, same sequence)."""

    def __init__(self, model, plan, states, null_pose, law, contact_params, horizon=100, dT=0.001,
                 tol_polish=1e-4, compiled=False, threads=8, cold_after_handover=True):
        """compiled: the rigid-body maps (centre of mass, the impedance-driven Euler steps) run the
        C restatement (blf_oracle_fbd.c) on `threads` threads instead of numpy (bench.py's
        configs[4] CPU baseline); the QP is the C oracle either way."""
        self.compiled, self.threads = compiled, threads
        self.model, self.N, self.dT = model, horizon, dT
        self.dt = float(plan["dt"])
        # integrate(0, T) with T = dt - dT: the reference schedule (FixedStepIntegrator.tpp:48-64)
        # integrates T + dT, so the robot advances exactly one knot per period (the device loop's
        # blf.closed_loop.period_final_time, restated)
        self.T = self.dt - dT
        self.law = law
        self.state = {k: np.array(v, dtype=np.float64) for k, v in states.items()
                      if k != "joint_torque"}
        self.null = null_pose
        C = len(model["frame_link"])
        self.cparams = np.tile(np.asarray(contact_params, np.float64), (C, 1))
        self.table = phase_table(plan)
        self.omega = plan["omega"]
        self.params = O.default_params(horizon, tol_polish=tol_polish, max_iter=100)   # blf/closed_loop.py MAX_ITER
        self.prev = None
        self.s = 0
        self.cold_after_handover = cold_after_handover

    def period(self):
        s, N = self.s, self.N
        omega = np.ascontiguousarray(self.omega[:, s:s + N])
        if self.compiled:
            com = O.fbd_com_batch(self.model, self.state)
            xi = com[:, :2] + com[:, 3:5] / omega[:, 0][:, None]
        else:
            com, xi = dcm_from_state(self.model, self.state, omega[:, 0])
        w = O.dcm_phase_expand(self.table, s, self.dt, N)
        w.update(xi_init=xi, omega=omega)
        pv, pl, ps = ((None, None, None) if self.prev is None else
                      (self.prev["vrp"], self.prev["lam"], self.prev["status"]))
        if ps is not None and self.cold_after_handover:
            # blf/closed_loop.py: a robot whose last window needed the interior point method starts cold
            ps = (ps | (self.prev["iters"] > 0)).astype(np.int32)
        pol = np.zeros(xi.shape[0], np.int32)
        # the window's QP and its warm start, kept for tests/golden/make_c5_windows.py
        self.last_window = dict(w, vrp_ws=pv, lam_ws=pl, prev_status=ps)
        st, xo, vrp, it, lam = O.dcm_mpc_solve_batch_warm(w, vrp_ws=pv, lam_ws=pl, shift=1, floor=1e-3,
                                                          params=self.params, threads=self.threads,
                                                          polished=pol, prev_status=ps)
        q_ref = posture_reference(self.law, com, vrp)
        C = len(self.model["frame_link"])
        if self.compiled:
            self.state = O.fbd_euler_impedance_batch(self.model, self.state, q_ref, self.law["kp"],
                                                     self.law["kd"], self.cparams, self.null, 0.0,
                                                     self.T, self.dT, threads=self.threads)
        for i in range(0 if self.compiled else xi.shape[0]):
            si = euler_integrate_impedance(self.model, self.state, i, q_ref[i], self.law["kp"],
                                           self.law["kd"], 0.0, self.T, self.dT,
                                           contacts=list(range(C)), contact_params=self.cparams,
                                           null_poses=self.null[i])
            for k in self.state:
                self.state[k][i] = si[k]
        self.prev = dict(vrp=vrp, lam=lam, status=st, iters=it)
        self.s = s + 1
        return dict(status=st, xi=xo, vrp=vrp, iters=it, lam=lam, polished=pol, com=com,
                    xi_init=xi, q_ref=q_ref)
