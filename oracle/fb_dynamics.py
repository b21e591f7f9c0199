"""TEST INFRASTRUCTURE ONLY — numpy restatement of FloatingBaseDynamicalSystem::dynamics
(src/System/src/FloatingBaseSystemDynamics.cpp:102-251) for the synthetic tree of
blf/robot.py, the checker of the blf_fbd_* kernels (tests/ only).

The reference takes M, h and the frame Jacobians from iDynTree KinDynComputations v1.1.0
(FloatingBaseSystemDynamics.cpp:163-206), which is absent here: the rigid-body terms are restated
from first principles in the MIXED representation iDynTree uses by default (base velocity =
(dp_B/dt, omega_B), both in world coordinates; frame velocities likewise):
  M = sum_l m_l Jv_l^T Jv_l + Jw_l^T (R_l Ic_l R_l^T) Jw_l         (Jv at the link COM)
  h = sum_l Jv_l^T m_l (a_l - g) + Jw_l^T (I_l alpha_l + w_l x I_l w_l)   with nu_dot = 0
and the reference's algebra after it (:193-248): known = -h + sum_c J_c^T w_c, known[6:] += tau,
nu_dot = LLT(M [+ reg]) \\ known.  Parity against iDynTree is therefore UNPINNED;
tests/test_fb_dynamics.py checks this oracle by self-consistency (symmetry / positive
definiteness of M, kinetic energy, nu^T h = 1/2 nu^T dM/dt nu + dV/dt, finite differences).
"""
import numpy as np

import oracle as O

G = np.array([0.0, 0.0, -9.81])


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def rot_axis(a, q):
    K = skew(a)
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * K @ K


PRISMATIC = 1   # model["joint_type"][j] (optional; absent: every joint revolute)


def prismatic(model):
    jt = model.get("joint_type")
    return np.zeros(model["n"], dtype=bool) if jt is None else np.asarray(jt) == PRISMATIC


def kinematics(model, base_pos, base_rot, joint_pos, base_vel, joint_vel):
    """World pose, mixed velocity and nu_dot = 0 bias acceleration of every link, plus the joint
    axes / origins in world coordinates.  A revolute joint rotates its child about z = R_P E a
    through the joint origin; a prismatic one (model["joint_type"][j] = 1, URDF "prismatic")
    translates it along z by q: r = R_P o + z q, w_c = w_P, v_c = v_P + w_P x r + z q_dot,
    a_c = a_P + al_P x r + w_P x (w_P x r) + 2 w_P x z q_dot (nu_dot = 0)."""
    n = model["n"]
    L = n + 1
    pri = prismatic(model)
    R = np.zeros((L, 3, 3)); p = np.zeros((L, 3))
    w = np.zeros((L, 3)); v = np.zeros((L, 3)); al = np.zeros((L, 3)); a = np.zeros((L, 3))
    z = np.zeros((n, 3)); o = np.zeros((n, 3))
    R[0], p[0], v[0], w[0] = base_rot, base_pos, base_vel[:3], base_vel[3:]
    for j in range(n):
        P, c = model["parent"][j], j + 1
        E = model["joint_rot"][j]
        z[j] = R[P] @ E @ model["joint_axis"][j]
        zs = z[j] * joint_vel[j]
        if pri[j]:
            R[c] = R[P] @ E
            r = R[P] @ model["joint_origin"][j] + z[j] * joint_pos[j]
            p[c] = p[P] + r
            o[j] = p[c]
            w[c] = w[P]
            v[c] = v[P] + np.cross(w[P], r) + zs
            al[c] = al[P]
            a[c] = a[P] + np.cross(al[P], r) + np.cross(w[P], np.cross(w[P], r)) + 2.0 * np.cross(w[P], zs)
            continue
        R[c] = R[P] @ E @ rot_axis(model["joint_axis"][j], joint_pos[j])
        r = R[P] @ model["joint_origin"][j]
        p[c] = p[P] + r
        o[j] = p[c]
        w[c] = w[P] + zs
        v[c] = v[P] + np.cross(w[P], r)
        al[c] = al[P] + np.cross(w[P], zs)
        a[c] = a[P] + np.cross(al[P], r) + np.cross(w[P], np.cross(w[P], r))
    return dict(R=R, p=p, w=w, v=v, al=al, a=a, z=z, o=o, pri=pri)


def ancestors(model):
    """anc[l] = joints on the path base -> link l."""
    n = model["n"]
    anc = [[] for _ in range(n + 1)]
    for j in range(n):
        anc[j + 1] = anc[model["parent"][j]] + [j]
    return anc


def point_jacobian(model, K, anc, l, x):
    """Mixed Jacobian (6 x (6+n)) of a point x rigidly attached to link l: (linear; angular)."""
    n = model["n"]
    J = np.zeros((6, 6 + n))
    J[:3, :3] = np.eye(3)
    J[:3, 3:6] = -skew(x - K["p"][0])
    J[3:, 3:6] = np.eye(3)
    for j in anc[l]:
        if K["pri"][j]:          # prismatic: the point moves along z, no rotation
            J[:3, 6 + j] = K["z"][j]
            continue
        J[:3, 6 + j] = np.cross(K["z"][j], x - K["o"][j])
        J[3:, 6 + j] = K["z"][j]
    return J


def mass_and_bias(model, K, gravity=G):
    n = model["n"]
    anc = ancestors(model)
    M = np.zeros((6 + n, 6 + n))
    h = np.zeros(6 + n)
    for l in range(n + 1):
        Rl = K["R"][l]
        c = K["p"][l] + Rl @ model["link_com"][l]
        rc = c - K["p"][l]
        J = point_jacobian(model, K, anc, l, c)
        Iw = Rl @ model["link_inertia"][l] @ Rl.T
        m = model["link_mass"][l]
        M += m * J[:3].T @ J[:3] + J[3:].T @ Iw @ J[3:]
        ac = K["a"][l] + np.cross(K["al"][l], rc) + np.cross(K["w"][l], np.cross(K["w"][l], rc))
        f = m * (ac - gravity)
        tq = Iw @ K["al"][l] + np.cross(K["w"][l], Iw @ K["w"][l])
        h += J[:3].T @ f + J[3:].T @ tq
    return M, h


def frame_state(model, K, f):
    """World transform (p, R), mixed velocity (v, w) and mixed Jacobian of frame f."""
    l = model["frame_link"][f]
    fp = model["frame_pose"][f]
    Rl, pl = K["R"][l], K["p"][l]
    pf = pl + Rl @ fp[:3]
    Rf = Rl @ fp[3:].reshape(3, 3)
    vel = np.concatenate([K["v"][l] + np.cross(K["w"][l], pf - pl), K["w"][l]])
    J = point_jacobian(model, K, ancestors(model), l, pf)
    return pf, Rf, vel, J


CONTACT_WRENCH = 1   # blf_fb_contacts.law: the caller's wrench instead of the continuous law


def dynamics(model, state, i, contacts=(), contact_params=None, null_poses=None, rho=0.01,
             reg=None, gravity=G, laws=None, wrenches=None):
    """FloatingBaseDynamicalSystem::dynamics for system i of a state batch.  contacts: frame
    indices; contact_params [C][4] (L, W, k, b); null_poses [C][12]; laws [C] (None: every
    contact a ContinuousContactModel) with wrenches [C][6], the (force, torque) a CONTACT_WRENCH
    contact's model returns (mapped through J_c^T like any ContactModel's wrench,
    FloatingBaseSystemDynamics.cpp:198-228).  Returns (base_acc[6], joint_acc[n], dpos[3],
    drot[3,3], djoint[n])."""
    s = {k: v[i] for k, v in state.items()}
    K = kinematics(model, s["base_pos"], s["base_rot"], s["joint_pos"], s["base_vel"], s["joint_vel"])
    M, h = mass_and_bias(model, K, gravity)
    known = -h
    for c, f in enumerate(contacts):
        pf, Rf, vel, J = frame_state(model, K, f)
        pose = np.concatenate([pf, Rf.reshape(-1)])
        if laws is not None and laws[c] == CONTACT_WRENCH:
            wrench = np.asarray(wrenches[c], dtype=np.float64)
        else:
            wrench = O.contact_eval(contact_params[c], vel, pose, null_poses[c])[0]
        known = known + J.T @ wrench
    known[6:] += s["joint_torque"]
    A = M + (reg if reg is not None else 0.0)
    L = np.linalg.cholesky(A)
    acc = np.linalg.solve(L.T, np.linalg.solve(L, known))
    dp, dR, dq = O.fbk_dynamics(rho, s["base_rot"], s["base_vel"], s["joint_vel"])
    return acc[:6], acc[6:], dp, dR, dq


def euler_integrate(model, state, i, t0, t1, dT, **kw):
    """ForwardEuler<FloatingBaseDynamicalSystem>::integrate(t0, t1) of system i with the
    FixedStepIntegrator schedule (iterations = ceil((t1 - t0)/dT), stale-time last step);
    returns the final state dict of that system."""
    s = {k: np.array(v[i], dtype=np.float64) for k, v in state.items()}
    iters = int(np.ceil((t1 - t0) / dT))
    steps = [dT] * (iters - 1)
    cur = t0 + dT * (iters - 2) if iters >= 2 else t0
    steps.append(t1 - cur)
    for h in steps:
        one = {k: v[None] for k, v in s.items()}
        ba, ja, dp, dR, dq = dynamics(model, one, 0, **kw)
        s["base_pos"] = s["base_pos"] + dp * h
        s["base_rot"] = s["base_rot"] + dR * h
        s["joint_pos"] = s["joint_pos"] + dq * h
        s["base_vel"] = s["base_vel"] + ba * h
        s["joint_vel"] = s["joint_vel"] + ja * h
    return s
