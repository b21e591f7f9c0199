"""BASELINE.json configs[4] on the device: the closed loop of the DCM-MPC planner and the
30-DoF floating-base robot with two ContinuousContactModel feet.

The reference has no closed-loop driver; a user of it alternates TimeVaryingDCMPlanner::advance()
(System/Advanceable.h:24-46) with ForwardEuler<FloatingBaseDynamicalSystem>::integrate
(System/include/BipedalLocomotion/System/ForwardEuler.tpp:18-49 over
System/src/FloatingBaseSystemDynamics.cpp:102-251, contact wrenches from
ContactModels/src/ContinuousContactModel.cpp:79-108) and writes the two maps between them.
One control period of this loop, stream-ordered on the device for a batch of robots:

  1. state -> plan:  xi = c_xy + cdot_xy / omega_0 from the robot's centre of mass
                     (blf_fb_dcm), the next window's xi_init;
  2. plan:           the window moved one knot (blf_dcm_mpc_solve_phased) and solved warm from the
                     previous period's solution (blf_dcm_mpc_solve_warm, shift 1);
  3. plan -> robot:  joint references from the plan's first VRP and the centre of mass, held over
                     the period (blf_dcm_posture_reference);
  4. robot:          ForwardEuler<FloatingBaseDynamicalSystem>::integrate(0, dt - dT) with a
                     joint impedance tracking them as the control input of every step
                     (blf_fbd_euler_integrate_impedance, contacts at the feet): the reference
                     schedule integrates T + dT (period_final_time), so the robot advances
                     exactly dt, one knot of the plan, per period.

The control period is the plan's knot spacing dt (the window moves one knot per period); the
impedance runs at the integration step dT (1 kHz): a 50 Hz zero-order hold of the joint
torques does not stabilise the robot's fast modes.  Every piece runs on the device; the host only
enqueues.
"""
import math

import numpy as np

from . import native
from . import robot as R


def fixed_step_schedule(t0, t1, dT):
    """The step sizes FixedStepIntegrator::integrate(t0, t1) takes (FixedStepIntegrator.tpp:48-64;
    blf_capi.hip step_schedule): iterations = ceil((t1 - t0) / dT), steps 0..iterations-2 of dT,
    the last one t1 - currentTime with the stale currentTime = t0 + dT (iterations - 2)."""
    iters = int(math.ceil((t1 - t0) / dT))
    cur = t0 + dT * (iters - 2) if iters >= 2 else t0
    return [dT] * (iters - 1) + [t1 - cur]


def period_final_time(dt, dT):
    """The final time T of integrate(0, T) that advances the robot by exactly one knot dt.

    With two or more iterations the reference schedule above integrates T + dT, not T: its last
    step runs from the START of the previous step (the stale currentTime).  integrate(0, dt) would
    therefore advance the robot dt + dT per period (21 ms at dt = 20 ms, dT = 1 ms) while the plan
    moves one 20 ms knot.  The loop keeps the reference call and its schedule, and asks for
    T = dt - dT: (iterations - 1) steps of dT and a last step of 2 dT (or iterations - 1 steps and
    a last dT when the quotient rounds up), dt in total."""
    T = dt - dT
    if not T > dT:
        raise ValueError(f"the control period {dt} needs at least two integration steps of {dT}")
    total = math.fsum(fixed_step_schedule(0.0, T, dT))
    assert abs(total - dt) <= 1e-12 * dt, (total, dt)
    return T

# ContinuousContactModel of each sole (length, width, spring_coeff, damper_coeff): the reference
# test's foot size; stiffness and damping for a 50 kg robot on two 0.12 x 0.09 m soles (about
# 1 cm of sink) that explicit Euler at dT = 1 ms integrates stably
CONTACT_PARAMS = (0.12, 0.09, 2.0e6, 2.0e4)
# The interior point iteration cap of the loop's plans (TimeVaryingDCMPlanner's "max_iterations";
# the solver default is 50).  A window the active-set start cannot certify -- an uncapturable DCM
# state, multipliers ~1e7 -- can need more from its warm start: tests/golden/c5_device_windows_r05.npz
# holds one that takes 92 (31 cold), on the device's trajectory of bench.py's loop.  Only such
# windows run that long; every other window stops at its certificate.
MAX_ITER = 100


class _nullcontext:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ClosedLoop:
    """A batch of robots, each closed around its own plan (problems.make_batch with the phase
    table), on one device.  `states` is a host dict (robot.standing_states), `plan` the host
    problem dict with a horizon of at least horizon + the number of periods to run."""

    def __init__(self, h, model, plan, states, horizon=100, dT=0.001, law=None,
                 contact_params=CONTACT_PARAMS, tol_polish=1e-4, stream=None, max_iter=MAX_ITER,
                 cold_after_handover=None):
        import torch
        self.h, self.N, self.dT, self.stream = h, horizon, dT, stream
        dev = torch.device("cuda", h.device)
        t = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(dev)
        self.dt = float(plan["dt"])
        self.T = period_final_time(self.dt, dT)      # integrate(0, T) advances the robot dt
        self.steps = fixed_step_schedule(0.0, self.T, dT)
        self.B = plan["omega"].shape[0]
        self.dm = h.fb_model(model)
        law = law if law is not None else R.posture_law_arrays(model)
        self.law = h.posture_law(law["q_nominal"], law["lean"])
        self.imp = h.joint_impedance(law["kp"], law["kd"])
        self.state = {k: t(states[k]) for k in native.FB_STATE_KEYS}
        C = len(model["frame_link"])
        self.contacts = dict(frame=t(np.arange(C), torch.int32),
                             params=t(np.tile(np.asarray(contact_params, np.float64), (C, 1))),
                             null_pose=t(R.sole_null_poses(model, states)))
        self.table = h.phase_table(t(plan["nphases"], torch.int32), t(plan["phase_begin"]),
                                   t(plan["phase_end"]), t(plan["phase_corners"]),
                                   t(plan["phase_ncorners"], torch.int32), ref=t(plan["phase_ref"]))
        self.omega = t(plan["omega"])
        self.params = native.default_params(horizon, max_facets=self.table["phase_b"].shape[2])
        self.params.tol_polish = tol_polish     # TimeVaryingDCMPlanner's warm-start trigger
        self.params.max_iter = max_iter         # (MAX_ITER: the uncapturable windows' iteration cap)
        self.params.dt = self.dt                # the knots of the plan are the QP's knots
        self.com = torch.empty((self.B, 6), dtype=torch.float64, device=dev)
        self.xi = torch.empty((self.B, 2), dtype=torch.float64, device=dev)
        self.q_ref = torch.empty((self.B, model["n"]), dtype=torch.float64, device=dev)
        self.bufs = [None, None]
        self.prev = None
        self.s = 0
        self.expand_path = False   # True: blf_dcm_phase_expand + blf_dcm_mpc_solve (A/B)
        # a robot whose last window needed the interior point method is planned cold: such windows
        # recur on the robot's next periods, and from a cold start the windows the warm kernel hands
        # over need 4.6 interior point iterations on average instead of 16.1 (DESIGN.md section 11,
        # tools/c5_handover_starts.py) -- stage 2 is on each group's critical path
        if cold_after_handover is None:   # BLF_C5_COLD_AFTER_HANDOVER=0: off (A/B)
            import os
            cold_after_handover = os.environ.get("BLF_C5_COLD_AFTER_HANDOVER", "1") != "0"
        self.cold_after_handover = cold_after_handover
        self.warm_status = torch.empty((self.B,), dtype=torch.int32, device=dev)
        self.dyn_events = None   # a list: period() appends (start, end) events of its dynamics launch

    def period(self):
        """One control period (stream-ordered; nothing synchronises).  Returns the plan."""
        h, s, N = self.h, self.s, self.N
        if s + N > self.omega.shape[1]:
            raise ValueError(f"the plan ends at knot {self.omega.shape[1]}; period {s} needs {s + N}")
        h.fb_dcm(self.dm, self.state, omega=self.omega, column=s, com=self.com, xi=self.xi,
                 stream=self.stream)
        warm = None
        if self.prev is not None:
            # a robot whose previous window was not solved (status != 0) is planned cold
            status = self.prev["status"]
            if self.cold_after_handover:   # status != 0 or iters > 0: start cold
                import torch
                with torch.cuda.stream(self.stream) if self.stream is not None else _nullcontext():
                    torch.bitwise_or(status, (self.prev["iters"] > 0).to(torch.int32), out=self.warm_status)
                status = self.warm_status
            warm = dict(vrp=self.prev["vrp"], lam=self.prev["lam"], shift=1, floor=1e-3,
                        status=status)
        if N <= 128 and not self.expand_path:   # the window read from the phase table
            out = h.dcm_mpc_solve_phased(self.table, s, self.xi, self.omega[:, s:s + N],
                                         self.params, warm=warm, out=self.bufs[s % 2],
                                         lambda_out=True, stream=self.stream)
        else:
            w = h.dcm_phase_expand(self.table, s, self.dt, N, stream=self.stream)
            w.update(xi_init=self.xi, omega=self.omega[:, s:s + N].contiguous())
            out = h.dcm_mpc_solve(w, self.params, out=self.bufs[s % 2], warm=warm,
                                  lambda_out=True, stream=self.stream)
        self.bufs[s % 2] = out
        h.posture_reference(self.law, self.com, out["vrp"], q_ref=self.q_ref, stream=self.stream)
        # integrate(0, T) with T = dt - dT: the reference schedule integrates T + dT, so the robot
        # advances exactly one knot dt per period, in step with the plan (period_final_time); the
        # dynamics are time-invariant, and a fixed interval keeps the step count the same in every
        # period
        ev = self.dyn_events
        if ev is not None:   # bench.py: HIP events around the dynamics launch, on this loop's stream
            import torch
            st = self.stream if self.stream is not None else torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
        h.fbd_euler_integrate_impedance(self.dm, self.state, self.imp, self.q_ref, 0.0, self.T,
                                        self.dT, contacts=self.contacts, stream=self.stream)
        if ev is not None:
            e1.record(st)
            ev.append((e0, e1))
        self.prev = out
        self.s = s + 1
        return out

def split_groups(h, model, plan, states, groups, horizon=100, **kw):
    """The robots of (plan, states) in `groups` contiguous groups, each a ClosedLoop on its own
    stream (one group: the current stream); the groups' kernels overlap on the device (the plan
    kernels' tails, a few QPs on an otherwise idle chip, run beside another group's dynamics).

    Every robot's periods are the same computation as in one ClosedLoop over all robots, bit for
    bit, when the QP launches of a group and of the whole batch pick the same kernels: the QP
    kernels choose their scan tree and the fused small-batch kernel by batch size
    (BLF_DPP_TREE_MAX_BATCH = 1024 and the fused kernel's limit, both for horizons <= 64 only).
    Horizons > 64 (the configs[4] loop's 100) are unaffected; with horizon <= 64, groups on the
    other side of those limits than the whole batch agree to rounding, not bit for bit."""
    import torch
    B = plan["omega"].shape[0]
    groups = max(1, min(int(groups), B))
    cut = [B * g // groups for g in range(groups + 1)]
    shared = ("knot_phase", "dt", "schedule")   # per-knot / scalar entries of the plan dict
    sl = lambda d, lo, hi: {k: (v if k in shared else v[lo:hi]) for k, v in d.items()}
    loops = []
    for g in range(groups):
        stream = torch.cuda.Stream(device=h.device) if groups > 1 else None
        loops.append(ClosedLoop(h, model, sl(plan, cut[g], cut[g + 1]), sl(states, cut[g], cut[g + 1]),
                                horizon=horizon, stream=stream, **kw))
    return loops
