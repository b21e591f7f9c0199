"""Synthetic floating-base robot models for the config-5 closed loop (BASELINE.json configs[4]:
"30-DoF": a 6-DoF floating base + 24 revolute joints).

The reference obtains the rigid-body terms from iDynTree KinDynComputations on a URDF model
(src/System/src/FloatingBaseSystemDynamics.cpp:163-206); neither iDynTree nor a robot description
ships here, so the model is a synthetic humanoid-like kinematic tree with randomised but physical
link masses and inertias (seeded).  Layout, consumed by blf_fbd_* (include/blf/blf_c.h) and by the
test oracle:

  parent       [n]      int32   parent LINK of joint j (link 0 = base); joint j moves link j + 1;
                                parent[j] <= j (topological order)
  joint_origin [n][3]           joint frame origin in the parent link frame
  joint_rot    [n][3][3]        fixed rotation parent link -> joint frame
  joint_axis   [n][3]           unit rotation axis in the joint frame (= child link frame at q=0)
  link_mass    [n+1]
  link_com     [n+1][3]         centre of mass in the link frame
  link_inertia [n+1][3][3]      rotational inertia about the COM, link frame (SPD)
  frame_link   [F]      int32   link a frame is attached to
  frame_pose   [F][12]          (p, R row-major) of the frame in its link frame
"""
import numpy as np

# (name, parent link name, origin in parent, axis) of the 24 joints
_TREE = [
    # left leg (hip yaw/roll/pitch, knee, ankle pitch/roll)
    ("l_hip_yaw", "base", (0.0, 0.09, -0.06), "z"), ("l_hip_roll", "l_hip_yaw", (0, 0, -0.03), "x"),
    ("l_hip_pitch", "l_hip_roll", (0, 0, 0), "y"), ("l_knee", "l_hip_pitch", (0, 0, -0.22), "y"),
    ("l_ankle_pitch", "l_knee", (0, 0, -0.22), "y"), ("l_ankle_roll", "l_ankle_pitch", (0, 0, 0), "x"),
    # right leg
    ("r_hip_yaw", "base", (0.0, -0.09, -0.06), "z"), ("r_hip_roll", "r_hip_yaw", (0, 0, -0.03), "x"),
    ("r_hip_pitch", "r_hip_roll", (0, 0, 0), "y"), ("r_knee", "r_hip_pitch", (0, 0, -0.22), "y"),
    ("r_ankle_pitch", "r_knee", (0, 0, -0.22), "y"), ("r_ankle_roll", "r_ankle_pitch", (0, 0, 0), "x"),
    # torso
    ("torso_pitch", "base", (0.0, 0.0, 0.08), "y"), ("torso_roll", "torso_pitch", (0, 0, 0.04), "x"),
    ("torso_yaw", "torso_roll", (0, 0, 0.04), "z"),
    # arms
    ("l_shoulder_pitch", "torso_yaw", (0.0, 0.14, 0.20), "y"),
    ("l_shoulder_roll", "l_shoulder_pitch", (0, 0.02, 0), "x"),
    ("l_shoulder_yaw", "l_shoulder_roll", (0, 0, -0.08), "z"), ("l_elbow", "l_shoulder_yaw", (0, 0, -0.10), "y"),
    ("r_shoulder_pitch", "torso_yaw", (0.0, -0.14, 0.20), "y"),
    ("r_shoulder_roll", "r_shoulder_pitch", (0, -0.02, 0), "x"),
    ("r_shoulder_yaw", "r_shoulder_roll", (0, 0, -0.08), "z"), ("r_elbow", "r_shoulder_yaw", (0, 0, -0.10), "y"),
    # neck
    ("neck_pitch", "torso_yaw", (0.0, 0.0, 0.26), "y"),
]
_AXES = {"x": (1.0, 0.0, 0.0), "y": (0.0, 1.0, 0.0), "z": (0.0, 0.0, 1.0)}


def _rotvec(v):
    th = np.linalg.norm(v)
    K = np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])
    if th == 0:
        return np.eye(3)
    return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K


def humanoid24(seed=2020):
    """The synthetic 6 + 24 DoF model used by config 5, with sole frames on both ankle-roll links."""
    rng = np.random.default_rng(seed)
    names = ["base"] + [t[0] for t in _TREE]
    n = len(_TREE)
    parent = np.array([names.index(t[1]) for t in _TREE], dtype=np.int32)
    joint_origin = np.array([t[2] for t in _TREE], dtype=np.float64)
    # small fixed mounting rotations so the joint frames are not all aligned with the parent
    joint_rot = np.stack([_rotvec(rng.normal(size=3) * 0.05) for _ in range(n)])
    joint_axis = np.array([_AXES[t[3]] for t in _TREE], dtype=np.float64)
    masses = rng.uniform(0.4, 3.0, n + 1)
    masses[0] = 8.0                                          # pelvis / base
    com = rng.normal(size=(n + 1, 3)) * 0.02
    inertia = np.zeros((n + 1, 3, 3))
    for l in range(n + 1):
        Q = _rotvec(rng.normal(size=3))
        d = rng.uniform(0.3, 1.0, 3) * masses[l] * 0.004
        d[2] = min(d[2], d[0] + d[1] - 1e-6)                 # triangle inequality of principal moments
        inertia[l] = Q @ np.diag(d) @ Q.T
    feet = [names.index("l_ankle_roll"), names.index("r_ankle_roll")]   # names index = link index
    frame_link = np.array(feet, dtype=np.int32)
    frame_pose = np.zeros((2, 12))
    for f in range(2):
        frame_pose[f, :3] = (0.02, 0.0, -0.06)
        frame_pose[f, 3:] = np.eye(3).reshape(-1)
    return dict(n=n, parent=parent, joint_origin=joint_origin, joint_rot=joint_rot,
                joint_axis=joint_axis, link_mass=masses, link_com=com, link_inertia=inertia,
                frame_link=frame_link, frame_pose=frame_pose, names=names)


REVOLUTE, PRISMATIC = 0, 1   # model["joint_type"] (blf_fb_model.joint_type; absent: all revolute)


def with_joint_types(model, prismatic=()):
    """A copy of `model` whose joints named (or indexed) in `prismatic` are prismatic: the child
    link slides along the joint axis by q instead of rotating about it (URDF "prismatic")."""
    names = list(model["names"])
    jt = np.zeros(model["n"], dtype=np.int32)
    for f in prismatic:
        jt[(names.index(f) - 1) if isinstance(f, str) else int(f)] = PRISMATIC
    out = dict(model)
    out["joint_type"] = jt
    return out


def reduce_fixed_joints(model, fixed):
    """The model with the joints in `fixed` (names or indices) removed, each fixed joint's child
    link merged into its parent link: what iDynTree's KinDynComputations does with a URDF's fixed
    joints, which carry no DoF (the reference's FloatingBaseSystemDynamics.cpp:53-74 sizes the
    state by the model's DoFs).  At q = 0 a joint's child frame sits at joint_origin with
    rotation joint_rot in its parent frame, so merging child c of joint j into parent P:
      mass m_P + m_c; COM (m_P c_P + m_c (o_j + E_j c_c)) / m; inertia about the new COM by the
      parallel-axis theorem (E_j I_c E_j^T + ...); every joint on c re-parented to P with origin
      o_j + E_j o_k and rotation E_j E_k (axes unchanged: they live in the joint frame); every
      frame on c moved to P with position o_j + E_j p and rotation E_j R.
    Fixed joints are merged deepest first (highest index), so chains of fixed joints collapse.
    The rigid-body terms of the result equal those of the full model with the fixed joints held at
    q = 0, q_dot = 0, their rows and columns removed (tests/test_fb_dynamics.py)."""
    n = int(model["n"])
    sizes = {"parent": n, "joint_origin": n, "joint_rot": n, "joint_axis": n, "link_mass": n + 1,
             "link_com": n + 1, "link_inertia": n + 1}
    for k, want in sizes.items():
        if len(model[k]) != want:
            raise ValueError(f"reduce_fixed_joints: {k} has {len(model[k])} entries, the model "
                             f"has {n} joints")
    if model.get("joint_type") is not None and len(model["joint_type"]) != n:
        raise ValueError("reduce_fixed_joints: joint_type must have one entry per joint")
    if len(model["frame_link"]) != len(model["frame_pose"]):
        raise ValueError("reduce_fixed_joints: frame_link and frame_pose differ in length")
    # the merge re-indexes joints and links in place, which assumes topological order
    for j, pj in enumerate(model["parent"]):
        if not 0 <= int(pj) <= j:
            raise ValueError(f"reduce_fixed_joints: joint {j} has parent link {int(pj)}; the joints "
                             f"must be in topological order (0 <= parent[j] <= j)")
    names = list(model["names"]) if "names" in model else None
    if names is None and any(isinstance(f, str) for f in fixed):
        raise ValueError("reduce_fixed_joints: joints named, but the model has no names")
    idx = sorted({(names.index(f) - 1) if isinstance(f, str) else int(f) for f in fixed}, reverse=True)
    n = model["n"]
    m = {k: (np.array(v, copy=True) if isinstance(v, np.ndarray) else v) for k, v in model.items()}
    parent = [int(x) for x in m["parent"]]
    o = [np.array(x, dtype=np.float64) for x in m["joint_origin"]]
    E = [np.array(x, dtype=np.float64) for x in m["joint_rot"]]
    ax = [np.array(x, dtype=np.float64) for x in m["joint_axis"]]
    mass = [float(x) for x in m["link_mass"]]
    com = [np.array(x, dtype=np.float64) for x in m["link_com"]]
    inertia = [np.array(x, dtype=np.float64) for x in m["link_inertia"]]
    flink = [int(x) for x in m["frame_link"]]
    jtype = [int(x) for x in m["joint_type"]] if m.get("joint_type") is not None else None
    fpose = [np.array(x, dtype=np.float64) for x in m["frame_pose"]]
    lnames = names if names is not None else [str(i) for i in range(n + 1)]
    S = lambda d: (d @ d) * np.eye(3) - np.outer(d, d)
    for j in idx:
        if not 0 <= j < len(parent):
            raise ValueError(f"reduce_fixed_joints: joint {j} out of range")
        c, P = j + 1, parent[j]
        cc = o[j] + E[j] @ com[c]                  # child COM in P's frame
        mt = mass[P] + mass[c]
        cn = (mass[P] * com[P] + mass[c] * cc) / mt if mt > 0 else com[P].copy()
        inertia[P] = (inertia[P] + mass[P] * S(com[P] - cn)
                      + E[j] @ inertia[c] @ E[j].T + mass[c] * S(cc - cn))
        mass[P], com[P] = mt, cn
        for k in range(len(parent)):               # joints on c move to P
            if parent[k] == c:
                parent[k] = P
                o[k] = o[j] + E[j] @ o[k]
                E[k] = E[j] @ E[k]
        for f in range(len(flink)):                # frames on c move to P
            if flink[f] == c:
                flink[f] = P
                Rf = fpose[f][3:].reshape(3, 3)
                fpose[f] = np.concatenate([o[j] + E[j] @ fpose[f][:3], (E[j] @ Rf).reshape(-1)])
        # drop joint j and link c; links above c shift down by one
        for lst in (o, E, ax) + ((jtype,) if jtype is not None else ()):
            del lst[j]
        del parent[j]
        for lst in (mass, com, inertia, lnames):
            del lst[c]
        parent = [x - 1 if x > c else x for x in parent]
        flink = [x - 1 if x > c else x for x in flink]
    nr = len(parent)
    out = dict(m)
    out.update(n=nr, parent=np.array(parent, dtype=np.int32), joint_origin=np.array(o).reshape(nr, 3),
               joint_rot=np.array(E).reshape(nr, 3, 3), joint_axis=np.array(ax).reshape(nr, 3),
               link_mass=np.array(mass), link_com=np.array(com), link_inertia=np.array(inertia),
               frame_link=np.array(flink, dtype=np.int32), frame_pose=np.array(fpose).reshape(-1, 12))
    if names is not None:
        out["names"] = lnames
    if jtype is not None:
        out["joint_type"] = np.array(jtype, dtype=np.int32)
    return out


def random_states(model, batch, seed=0, spread=0.3):
    """Batch of floating-base states near a standing pose: base at 0.75 m, joints within
    +-spread rad, velocities ~N(0, 0.5)."""
    rng = np.random.default_rng(seed)
    n = model["n"]
    base_rot = np.stack([_rotvec(rng.normal(size=3) * 0.1) for _ in range(batch)])
    return dict(
        base_vel=rng.normal(size=(batch, 6)) * 0.5,
        joint_vel=rng.normal(size=(batch, n)) * 0.5,
        base_pos=np.column_stack([rng.normal(size=(batch, 2)) * 0.01, np.full(batch, 0.75)]),
        base_rot=base_rot,
        joint_pos=rng.uniform(-spread, spread, (batch, n)),
        joint_torque=rng.normal(size=(batch, n)) * 5.0,
    )


# ---- config 5 closed loop: a standing start (synthetic input generation, host side) -----------
def sole_offsets(model):
    """Positions of the sole frames relative to the base origin at the nominal posture (all joints
    0, base orientation identity): plain forward kinematics of the tree's fixed transforms."""
    n = model["n"]
    Rl = [np.eye(3)] + [None] * n
    pl = [np.zeros(3)] + [None] * n
    for j in range(n):
        P = model["parent"][j]
        Rl[j + 1] = Rl[P] @ model["joint_rot"][j]
        pl[j + 1] = pl[P] + Rl[P] @ model["joint_origin"][j]
    out = []
    for f in range(len(model["frame_link"])):
        l = model["frame_link"][f]
        out.append(pl[l] + Rl[l] @ model["frame_pose"][f, :3])
    return np.array(out)


def standing_states(model, batch, seed=0, spread=0.05, vel=0.02):
    """Batch of states near the nominal standing posture: base upright at the height that puts the
    soles on z = 0 with straight legs, the torso, arm and neck joints within +-spread rad of 0,
    small velocities.  (Random leg joints would start the soles off the ground or in it: the
    contact springs then kick the robot at the first step.)"""
    rng = np.random.default_rng(seed)
    n = model["n"]
    h = -sole_offsets(model)[:, 2].mean()
    legs = np.array([nm[0] in "lr" and nm[1] == "_" and nm[2:].split("_")[0] in ("hip", "knee", "ankle")
                     for nm in model["names"][1:]])
    q = rng.uniform(-spread, spread, (batch, n))
    q[:, legs] = 0.0
    return dict(
        base_vel=rng.normal(size=(batch, 6)) * vel,
        joint_vel=rng.normal(size=(batch, n)) * vel,
        base_pos=np.column_stack([rng.normal(size=(batch, 2)) * 0.01, np.full(batch, h)]),
        base_rot=np.broadcast_to(np.eye(3), (batch, 3, 3)).copy(),
        joint_pos=q,
    )


def sole_null_poses(model, states):
    """ContinuousContactModel null-force transforms [B][F][12] of the sole frames: each foot's
    nominal sole position under the base on the ground (z = 0), orientation identity."""
    off = sole_offsets(model)
    B, F = states["base_pos"].shape[0], off.shape[0]
    null = np.zeros((B, F, 12))
    null[:, :, 0] = states["base_pos"][:, None, 0] + off[None, :, 0]
    null[:, :, 1] = states["base_pos"][:, None, 1] + off[None, :, 1]
    null[:, :, 3:] = np.eye(3).reshape(-1)
    return null


def joint_inertias(model):
    """Composite inertia of every joint's subtree about the joint axis at the nominal posture
    (joints 0, base identity): sum over the subtree's links of z^T R I_c R^T z + m |z x (c - o)|^2."""
    n = model["n"]
    Rl = [np.eye(3)] + [None] * n
    pl = [np.zeros(3)] + [None] * n
    z, o = np.zeros((n, 3)), np.zeros((n, 3))
    for j in range(n):
        P = model["parent"][j]
        Rl[j + 1] = Rl[P] @ model["joint_rot"][j]
        pl[j + 1] = pl[P] + Rl[P] @ model["joint_origin"][j]
        z[j], o[j] = Rl[j + 1] @ model["joint_axis"][j], pl[j + 1]
    anc = [set() for _ in range(n + 1)]
    for j in range(n):
        anc[j + 1] = anc[model["parent"][j]] | {j}
    I = np.zeros(n)
    for l in range(n + 1):
        c = pl[l] + Rl[l] @ model["link_com"][l]
        Iw = Rl[l] @ model["link_inertia"][l] @ Rl[l].T
        for j in anc[l]:
            r = np.cross(z[j], c - o[j])
            I[j] += z[j] @ Iw @ z[j] + model["link_mass"][l] * (r @ r)
    return I


def posture_law_arrays(model, freq=20.0, zeta=1.0, ankle_inertia=0.2, hip_lean=0.0, gravity=9.81):
    """The closed loop's plan -> robot map: joint references (blf_dcm_posture_reference) tracked
    by a joint impedance (blf_fbd_euler_integrate_impedance), PD to the zero posture with
    per-joint gains for one natural frequency (kp = freq^2 I_j, I_j the joint's composite
    inertia; kd = 2 zeta sqrt(kp I_j), damped for the joint's own subtree, so explicit Euler
    sees a bounded freq * dT on every joint).  The plan enters through the ankles: the ankle
    pitch / roll references move by m g / (2 kp_ankle) rad per metre of (r0 - c), the offset at
    which each foot's ankle impedance exerts the torque m g / 2 (r0 - c) that moves the centre of
    pressure from under the centre of mass to the planned VRP; the hips can counter-lean the
    trunk (hip_lean rad per metre).  The ankles carry the body in stance, so their inertia is
    floored at `ankle_inertia` (the free foot alone would give them far too weak a posture)."""
    n = model["n"]
    names = model["names"][1:]   # joint j moves link j + 1
    I = joint_inertias(model)
    Ik = I.copy()
    for side in ("l", "r"):
        for jn in ("ankle_pitch", "ankle_roll"):
            j = names.index(f"{side}_{jn}")
            Ik[j] = max(I[j], ankle_inertia)
    kp = freq * freq * Ik
    mg2 = 0.5 * model["link_mass"].sum() * gravity
    L = np.zeros((n, 2))
    for side in ("l", "r"):
        jp, jr = names.index(f"{side}_ankle_pitch"), names.index(f"{side}_ankle_roll")
        L[jp, 0] = mg2 / kp[jp]
        L[jr, 1] = -mg2 / kp[jr]
        L[names.index(f"{side}_hip_pitch"), 0] = -hip_lean
        L[names.index(f"{side}_hip_roll"), 1] = hip_lean
    return dict(q_nominal=np.zeros(n), lean=L, kp=kp, kd=2.0 * zeta * np.sqrt(kp * I))
