"""Synthetic batched DCM-MPC workloads (SURVEY.md 8(d) "Synthetic inputs").

Footstep plans -> contact lists (one per foot) -> contact phases -> per-knot support-polygon
corner sets, plus the DCM references and the time-varying omega.  The phase sweep is the
reference's ContactPhaseList::createPhases (src/Planners/src/ContactPhaseList.cpp:16-84); the
per-knot phase rule is `begin <= t_k < end`, and every contact time is an integer knot index
times dt (computed as `index * dt` in fp64) so knot/phase ties are exact and reproducible.

Everything here is host-side input preparation; the support-polygon H-rep of each corner set
is produced on the device by blf_hull2d_hrep (blf.native.hull2d_hrep).
"""
import numpy as np

FOOT_LENGTH = 0.12   # ContinousContactModelTest.cpp:46-47 values (L, W)
FOOT_WIDTH = 0.09
DS_KNOTS = 10        # double support 0.2 s at dt = 0.02
SS_KNOTS = 30        # single support 0.6 s
GRAVITY = 9.81
SEED = 20201015


def contact_schedule(n_footsteps, horizon, first_ds=DS_KNOTS):
    """Knot-index schedule of the plan: returns {foot: [(act_knot, deact_knot, pose_slot)]}.

    Footsteps 0 and 1 are the initial left/right stance (active from knot 0); step j >= 0 swings
    the right foot for even j, the left foot for odd j: lift at first_ds + 40 j, land at
    first_ds + 30 + 40 j (first_ds = 10: the standard 0.2 s double support; longer: the robot
    stands first, as the config-5 closed loop does).  The last contact of each foot stays active
    until past the horizon.
    """
    assert n_footsteps >= 2
    lists = {"left": [], "right": []}
    act = {"left": 0, "right": 0}
    slot = {"left": 0, "right": 1}
    nxt = 2
    for j in range(n_footsteps - 2):
        foot = "right" if j % 2 == 0 else "left"
        lift = first_ds + (DS_KNOTS + SS_KNOTS) * j
        land = lift + SS_KNOTS
        lists[foot].append((act[foot], lift, slot[foot]))
        act[foot], slot[foot] = land, nxt
        nxt += 1
    last = max(horizon, max(act.values())) + 100
    for foot in ("left", "right"):
        lists[foot].append((act[foot], last, slot[foot]))
    return lists


def phases_from_schedule(lists, dt):
    """ContactPhaseList::createPhases over the two foot lists (times = knot * dt)."""
    names = ["left", "right"]   # std::map<std::string, ContactList> iteration order
    acts, deacts = {}, {}
    for li, name in enumerate(names):
        for ci, (a, d, _) in enumerate(lists[name]):
            acts.setdefault(a * dt, []).append((li, ci))
            deacts.setdefault(d * dt, []).append((li, ci))
    ta, td = sorted(acts), sorted(deacts)
    cur = {}
    for (li, ci) in acts[ta[0]]:
        cur[li] = ci
    begin, ia, id_ = ta[0], 1, 0
    phases = []
    while (len(ta) - ia) + (len(td) - id_) > 1:
        if ia == len(ta) or td[id_] <= ta[ia]:
            t = td[id_]
            phases.append((begin, t, dict(cur)))
            begin = t
            for (li, _) in deacts[t]:
                cur.pop(li, None)
            id_ += 1
            if ia < len(ta) and id_ < len(td) and td[id_] == ta[ia]:
                for (li, ci) in acts[ta[ia]]:
                    cur.setdefault(li, ci)
                ia += 1
        else:
            t = ta[ia]
            phases.append((begin, t, dict(cur)))
            begin = t
            for (li, ci) in acts[t]:
                cur.setdefault(li, ci)
            ia += 1
    phases.append((begin, td[id_], dict(cur)))
    return phases


def rectangle_corners(pose):
    """pose [..., 3] = (x, y, yaw) -> corners [..., 4, 2] = pose * (+-L/2, +-W/2)."""
    x, y, yaw = pose[..., 0], pose[..., 1], pose[..., 2]
    c, s = np.cos(yaw), np.sin(yaw)
    out = []
    for sx in (0.5, -0.5):
        for sy in (0.5, -0.5):
            px, py = sx * FOOT_LENGTH, sy * FOOT_WIDTH
            out.append(np.stack([x + c * px - s * py, y + s * px + c * py], axis=-1))
    return np.stack(out, axis=-2)


def make_batch(batch, horizon=100, n_footsteps=6, dt=0.02, seed=SEED, start=0, first_ds=DS_KNOTS):
    """Problems [start, start+batch) of the synthetic workload with the given seed.

    Problem i's random draws depend only on (seed, start + i), so shards are reproducible.
    first_ds: knots of the initial double support (contact_schedule).
    """
    F = n_footsteps
    rows = np.arange(start, start + batch, dtype=np.uint64)
    # per-problem Philox streams keyed by the global problem index
    R = max(F, 3)
    draws = np.empty((batch, R, 6))
    for r, gi in enumerate(rows):
        rng = np.random.Generator(np.random.Philox(key=[seed, int(gi)]))
        draws[r] = rng.random((R, 6))
    u = draws * 2.0 - 1.0                                       # U(-1, 1)
    poses = np.zeros((batch, F, 3))
    poses[:, 0] = np.stack([np.zeros(batch), 0.10 + 0.02 * u[:, 0, 0], 0.1 * u[:, 0, 1]], -1)
    poses[:, 1] = np.stack([np.zeros(batch), -0.10 + 0.02 * u[:, 1, 0], 0.1 * u[:, 1, 1]], -1)
    x = np.zeros(batch)
    for j in range(F - 2):
        x = x + 0.20 + 0.05 * u[:, j + 2, 2]
        side = -1.0 if j % 2 == 0 else 1.0                       # right foot first
        poses[:, j + 2] = np.stack([x, side * 0.10 + 0.02 * u[:, j + 2, 0], 0.1 * u[:, j + 2, 1]], -1)

    lists = contact_schedule(F, horizon, first_ds)
    phases = phases_from_schedule(lists, dt)
    corners_all = rectangle_corners(poses)                      # [B, F, 4, 2]
    foot_names = ["left", "right"]
    # the phase table: each phase's active-contact corners (sorted by list name) and centroid
    NP = len(phases)
    ph_corners = np.zeros((batch, NP, 8, 2))
    ph_ncorners = np.zeros((batch, NP), dtype=np.int32)
    for pi, (b0, e0, act) in enumerate(phases):
        slots = [lists[foot_names[li]][ci][2] for li, ci in sorted(act.items())]
        pts = np.concatenate([corners_all[:, sl] for sl in slots], axis=1)
        ph_corners[:, pi, :pts.shape[1]] = pts
        ph_ncorners[:, pi] = pts.shape[1]
    ph_ref = ph_corners.sum(axis=2) / ph_ncorners[:, :, None].astype(np.float64)
    # knot -> phase: begin <= t_k < end (t_k = k dt)
    knot_phase = np.full(horizon + 1, -1, dtype=np.int32)
    for k in range(horizon + 1):
        t = k * dt
        for pi, (b0, e0, act) in enumerate(phases):
            if b0 <= t < e0:
                knot_phase[k] = pi
                break
        assert knot_phase[k] >= 0, "knot outside every contact phase"
    corners = np.ascontiguousarray(ph_corners[:, knot_phase])
    ncorners = np.ascontiguousarray(ph_ncorners[:, knot_phase])
    centroid = np.ascontiguousarray(ph_ref[:, knot_phase])
    phi = 2.0 * np.pi * draws[:, 0, 5]
    z = 0.53 + 0.02 * np.sin(2.0 * np.pi * np.arange(horizon)[None, :] / horizon + phi[:, None])
    omega = np.sqrt(GRAVITY / z)
    noise = np.stack([draws[:, 1, 5] - 0.5, draws[:, 2, 5] - 0.5], -1) * 0.02
    xi_init = centroid[:, 0] + noise
    return dict(
        xi_init=np.ascontiguousarray(xi_init),
        omega=np.ascontiguousarray(omega),
        xi_ref=np.ascontiguousarray(centroid),
        vrp_ref=np.ascontiguousarray(centroid[:, :horizon]),
        corners=np.ascontiguousarray(corners),
        ncorners=np.ascontiguousarray(ncorners),
        poses=poses,
        knot_phase=knot_phase,
        nphases=np.full(batch, NP, dtype=np.int32),
        phase_begin=np.ascontiguousarray(np.broadcast_to([p[0] for p in phases], (batch, NP))),
        phase_end=np.ascontiguousarray(np.broadcast_to([p[1] for p in phases], (batch, NP))),
        phase_corners=ph_corners,
        phase_ncorners=ph_ncorners,
        phase_ref=np.ascontiguousarray(ph_ref),
        dt=dt,
        schedule=lists,
    )


def swing_splines(prob, apex_height=0.05, queries=32):
    """Quintic swing-foot splines for every swing of every problem.

    Each swing (lift -> land of one foot) is a 3-knot spline (lift, mid, land) in x, y, z with
    zero velocity/acceleration at lift and land; the apex knot sits at the mid time, halfway in
    x/y, at apex_height in z, with the average x/y velocity and zero z velocity.
    Returns knots_t [S, 3], knots_pva [S, 3, 3, 3], tq [S, Q] (uniform in [lift, land]).
    """
    lists, dt, poses = prob["schedule"], prob["dt"], prob["poses"]
    B = poses.shape[0]
    kt, kp, tq = [], [], []
    for foot in ("left", "right"):
        lst = lists[foot]
        for (a0, d0, s0), (a1, _, s1) in zip(lst[:-1], lst[1:]):
            t0, t1 = d0 * dt, a1 * dt
            tm = 0.5 * (t0 + t1)
            p0, p1 = poses[:, s0, :2], poses[:, s1, :2]
            pva = np.zeros((B, 3, 3, 3))
            pva[:, 0, 0, :2] = p0
            pva[:, 2, 0, :2] = p1
            pva[:, 1, 0, :2] = 0.5 * (p0 + p1)
            pva[:, 1, 0, 2] = apex_height
            pva[:, 1, 1, :2] = (p1 - p0) / (t1 - t0)
            kt.append(np.broadcast_to(np.array([t0, tm, t1]), (B, 3)))
            kp.append(pva)
            tq.append(np.broadcast_to(np.linspace(t0, t1, queries), (B, queries)))
    return (np.ascontiguousarray(np.concatenate(kt)), np.ascontiguousarray(np.concatenate(kp)),
            np.ascontiguousarray(np.concatenate(tq)))


def window(full, start, horizon, xi_init=None):
    """Receding-horizon window [start, start + horizon) of a longer plan (make_batch with a
    horizon of at least start + horizon): the per-knot arrays of knots start.., the references of
    knots start..start+horizon, and xi_init (default: the plan's).  Works on numpy arrays and on
    device tensors alike (the A, b, nfacets keys are sliced when present)."""
    s, N = start, horizon
    out = {"xi_init": full["xi_init"] if xi_init is None else xi_init}
    for k in ("omega", "vrp_ref", "A", "b", "nfacets"):
        if k in full:
            out[k] = full[k][:, s:s + N]
    out["xi_ref"] = full["xi_ref"][:, s:s + N + 1]
    for k in list(out):
        v = out[k]
        out[k] = v.contiguous() if hasattr(v, "contiguous") else np.ascontiguousarray(v)
    return out


# The phases of the reference's ContactPhaseList test (src/Planners/tests/ContactPhaseListTest.cpp
# :15-153; tests/golden/contact_phases.json): (begin, end, contact index per list or -1), lists in
# std::map order (additional, left, right).  Phases [4, 5) and [6, 7) have three contacts.
REFERENCE_THREE_CONTACT_PHASES = (
    (0.0, 1.0, (-1, 0, 0)), (1.0, 2.0, (-1, -1, 0)), (2.0, 3.0, (-1, 1, 0)), (3.0, 4.0, (-1, 1, -1)),
    (4.0, 5.0, (0, 1, 1)), (5.0, 6.0, (-1, -1, 1)), (6.0, 7.0, (1, 2, 1)), (7.0, 7.5, (1, -1, -1)))


def three_contact_plan(batch, dt=0.1, knots=75, seed=SEED, xi_offset=0.05,
                       phases=REFERENCE_THREE_CONTACT_PHASES):
    """Plans over three contact lists (bench.py --workload mc; tests/multi_contact.py builds the same
    plans from the oracle's createPhases): standing with the feet turned out and a hand support
    ahead, so a phase with all three contacts has a hull of up to 9 facets (max_facets 16).  Each
    contact is a 0.12 x 0.09 m rectangle; returns make_batch's phase-table keys plus omega,
    xi_init (the first phase's centroid plus a uniform offset) and dt."""
    begin = np.array([p[0] for p in phases])
    end = np.array([p[1] for p in phases])
    active = np.array([p[2] for p in phases], dtype=np.int64)
    NP = len(phases)
    rng = np.random.default_rng(seed)
    corners = np.zeros((batch, NP, 16, 2))
    ncorners = np.zeros((batch, NP), dtype=np.int32)
    for q in range(batch):
        u = rng.uniform(-1.0, 1.0, (3, 4, 3))
        pose = np.zeros((3, 4, 3))      # [list][contact][x, y, yaw]
        for c in range(4):
            pose[1, c] = (0.005 * u[1, c, 0], 0.14 + 0.005 * u[1, c, 1], 1.50 + 0.03 * u[1, c, 2])
            pose[2, c] = (0.005 * u[2, c, 0], -0.14 + 0.005 * u[2, c, 1], -0.03 + 0.03 * u[2, c, 2])
            pose[0, c] = (0.19 + 0.005 * u[0, c, 0], 0.005 * u[0, c, 1], 0.85 + 0.03 * u[0, c, 2])
        for p in range(NP):
            pts = [rectangle_corners(pose[l, active[p, l]]) for l in range(3) if active[p, l] >= 0]
            if pts:
                pts = np.concatenate(pts)
                corners[q, p, :len(pts)] = pts
                ncorners[q, p] = len(pts)
    ref = corners.sum(axis=2) / np.maximum(ncorners, 1)[..., None]
    k = np.arange(knots)
    z = 0.53 + 0.01 * np.sin(2.0 * np.pi * k / knots)[None, :] * np.ones((batch, 1))
    omega = np.sqrt(GRAVITY / z)
    xi_init = ref[:, 0] + rng.uniform(-xi_offset, xi_offset, (batch, 2))
    return dict(nphases=np.full(batch, NP, dtype=np.int32),
                phase_begin=np.ascontiguousarray(np.broadcast_to(begin, (batch, NP))),
                phase_end=np.ascontiguousarray(np.broadcast_to(end, (batch, NP))),
                phase_corners=corners, phase_ncorners=ncorners, phase_ref=ref,
                omega=np.ascontiguousarray(omega), xi_init=xi_init, dt=dt)
