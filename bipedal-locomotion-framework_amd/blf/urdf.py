"""URDF -> the floating-base model layout of blf/robot.py (consumed by blf_fb_model / blf_fbd_*).

The reference's FloatingBaseDynamicalSystem takes an iDynTree model
(src/System/src/FloatingBaseSystemDynamics.cpp:53-74, setRobotModel), which a user loads from a
URDF with iDynTree's ModelLoader (optionally reduced to a list of "considered joints", the others
locked).  iDynTree is not in this image; this module is the same path for the device kernels:

  * links and joints from the URDF XML (standard library parser, nothing executed from the file);
  * the tree rooted at the floating base (the one link that is no joint's child, or `base=`),
    joints numbered in depth-first preorder, children in document order -- so parent[j] <= j and
    every subtree is a contiguous run of joints, the order the dynamics kernel's prefix-sum
    subtree sums use (csrc/fb_dynamics.hip build_topo);
  * joint j: origin xyz -> joint_origin, rpy -> joint_rot (R = Rz(y) Ry(p) Rx(r), the child frame
    in the parent frame), axis -> joint_axis (normalised; URDF default x);
    "revolute" / "continuous" -> revolute, "prismatic" -> prismatic, "fixed" and every joint not in
    `considered_joints` -> merged into its parent link (robot.reduce_fixed_joints, what iDynTree does
    with DoF-less joints); "floating" / "planar" joints inside the tree are refused;
  * link inertials: origin xyz -> link_com, inertia about the COM in the inertial frame rotated into
    the link frame (R I R^T); a link without <inertial> is massless;
  * `frames`: link names exposed as frames (e.g. the soles, usually massless links on fixed
    joints): frame f sits at the origin of its link, and follows the merge onto the link that
    carries it.
"""
import xml.etree.ElementTree as ET

import numpy as np

from . import robot

_MOVING = {"revolute": robot.REVOLUTE, "continuous": robot.REVOLUTE, "prismatic": robot.PRISMATIC}


def rpy_matrix(rpy):
    """URDF's fixed-axis roll, pitch, yaw: R = Rz(yaw) Ry(pitch) Rx(roll)."""
    r, p, y = (float(v) for v in rpy)
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rx = np.array([[1.0, 0.0, 0.0], [0.0, cr, -sr], [0.0, sr, cr]])
    Ry = np.array([[cp, 0.0, sp], [0.0, 1.0, 0.0], [-sp, 0.0, cp]])
    Rz = np.array([[cy, -sy, 0.0], [sy, cy, 0.0], [0.0, 0.0, 1.0]])
    return Rz @ Ry @ Rx


def _vec(el, attr, default):
    if el is None or el.get(attr) is None:
        return np.array(default, dtype=np.float64)
    v = np.array([float(t) for t in el.get(attr).split()], dtype=np.float64)
    if v.shape != (3,):
        raise ValueError(f"load_urdf: {attr}=\"{el.get(attr)}\" is not three numbers")
    return v


def _inertial(link):
    """(mass, COM in the link frame, inertia about the COM in the link frame) of a <link>."""
    ine = link.find("inertial")
    if ine is None:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    org = ine.find("origin")
    com = _vec(org, "xyz", (0.0, 0.0, 0.0))
    R = rpy_matrix(_vec(org, "rpy", (0.0, 0.0, 0.0)))
    m_el = ine.find("mass")
    mass = float(m_el.get("value")) if m_el is not None else 0.0
    i_el = ine.find("inertia")
    I = np.zeros((3, 3))
    if i_el is not None:
        g = lambda k: float(i_el.get(k, 0.0))
        I = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")],
                      [g("ixz"), g("iyz"), g("izz")]])
    if mass < 0.0:
        raise ValueError(f"load_urdf: link {link.get('name')} has a negative mass")
    return mass, com, R @ I @ R.T


def load_urdf(source, frames=(), base=None, considered_joints=None):
    """The model dict of blf/robot.py from a URDF file path or XML string.

    frames            link names to expose as frames (frame_link / frame_pose), in this order
    base              the floating base link (default: the tree's root)
    considered_joints joint names kept as degrees of freedom (default: every moving joint); the
                      other joints are locked at q = 0, as iDynTree's reduced model loader does,
                      and the degrees of freedom follow the list's order, as iDynTree orders them
                      (the list must name every joint after its parent's: the kernels need
                      parent[j] <= j; otherwise ValueError).  Without it: depth-first preorder.
    """
    text = source if isinstance(source, str) and source.lstrip().startswith("<") else open(source).read()
    root = ET.fromstring(text)
    if root.tag != "robot":
        raise ValueError("load_urdf: the document's root element is not <robot>")
    links = {}
    for l in root.findall("link"):
        if l.get("name") in links:
            raise ValueError(f"load_urdf: link {l.get('name')} is defined twice")
        links[l.get("name")] = l
    kids = {name: [] for name in links}
    parent_joint = {}
    for j in root.findall("joint"):
        pl, cl = j.find("parent").get("link"), j.find("child").get("link")
        if pl not in links or cl not in links:
            raise ValueError(f"load_urdf: joint {j.get('name')} connects an undefined link")
        if cl in parent_joint:
            raise ValueError(f"load_urdf: link {cl} is the child of two joints (not a tree)")
        parent_joint[cl] = j
        kids[pl].append(j)
    roots = [name for name in links if name not in parent_joint]
    if base is None:
        if len(roots) != 1:
            raise ValueError(f"load_urdf: the links form {len(roots)} trees ({roots}); one expected")
        base = roots[0]
    elif base not in links:
        raise ValueError(f"load_urdf: base link {base} is not in the model")
    if parent_joint.get(base) is not None:
        raise ValueError("load_urdf: a base below the tree's root (re-rooting) is not supported")
    # joints in depth-first preorder from the base, children in document order
    order, stack = [], [base]
    link_index = {base: 0}
    while stack:
        lk = stack.pop()
        for j in reversed(kids[lk]):
            stack.append(j.find("child").get("link"))
        if lk != base:
            order.append(parent_joint[lk])
            link_index[lk] = len(order)
    unreached = [name for name in links if name not in link_index]
    if unreached:
        raise ValueError(f"load_urdf: links not connected to the base: {unreached}")
    n = len(order)
    names = [base] + [j.get("name") for j in order]
    parent = np.zeros(n, dtype=np.int32)
    joint_origin = np.zeros((n, 3))
    joint_rot = np.zeros((n, 3, 3))
    joint_axis = np.zeros((n, 3))
    joint_type = np.zeros(n, dtype=np.int32)
    fixed = []
    for k, j in enumerate(order):
        typ = j.get("type")
        if typ not in _MOVING and typ != "fixed":
            raise ValueError(f"load_urdf: joint {j.get('name')} of type {typ} is not supported "
                             "(revolute, continuous, prismatic, fixed)")
        parent[k] = link_index[j.find("parent").get("link")]
        org = j.find("origin")
        joint_origin[k] = _vec(org, "xyz", (0.0, 0.0, 0.0))
        joint_rot[k] = rpy_matrix(_vec(org, "rpy", (0.0, 0.0, 0.0)))
        ax = _vec(j.find("axis"), "xyz", (1.0, 0.0, 0.0))
        na = np.linalg.norm(ax)
        if typ != "fixed" and not na > 0.0:
            raise ValueError(f"load_urdf: joint {j.get('name')} has a zero axis")
        joint_axis[k] = ax / na if na > 0.0 else (1.0, 0.0, 0.0)
        joint_type[k] = _MOVING.get(typ, robot.REVOLUTE)
        if typ == "fixed" or (considered_joints is not None and j.get("name") not in considered_joints):
            fixed.append(k)
    if considered_joints is not None:
        missing = [c for c in considered_joints if c not in names[1:]]
        if missing:
            raise ValueError(f"load_urdf: considered joints not in the model: {missing}")
    link_names = [base] + [j.find("child").get("link") for j in order]
    inert = [_inertial(links[name]) for name in link_names]
    frame_link, frame_pose = [], []
    for f in frames:
        if f not in link_index:
            raise ValueError(f"load_urdf: frame {f} is not a link of the model")
        frame_link.append(link_index[f])
        frame_pose.append(np.concatenate([np.zeros(3), np.eye(3).reshape(-1)]))
    model = dict(n=n, parent=parent, joint_origin=joint_origin, joint_rot=joint_rot,
                 joint_axis=joint_axis,
                 link_mass=np.array([m for m, _, _ in inert]),
                 link_com=np.array([c for _, c, _ in inert]),
                 link_inertia=np.array([I for _, _, I in inert]),
                 frame_link=np.array(frame_link, dtype=np.int32),
                 frame_pose=np.array(frame_pose, dtype=np.float64).reshape(-1, 12),
                 names=names)
    if (joint_type != robot.REVOLUTE).any():
        model["joint_type"] = joint_type
    if fixed:
        model = robot.reduce_fixed_joints(model, fixed)
    if considered_joints is not None:
        wanted = [c for c in dict.fromkeys(considered_joints) if c in model["names"][1:]]
        if wanted != list(model["names"][1:]):
            model = reorder_joints(model, [model["names"].index(c) - 1 for c in wanted])
    return model


def reorder_joints(model, perm):
    """The model with its joints in the order perm (perm[k] = the joint placed at k, with its child
    link): every joint / link array permuted, parents and frame links re-indexed.  ValueError when
    a joint would precede its parent's joint (the kernels need parent[j] <= j)."""
    n = model["n"]
    perm = [int(o) for o in perm]
    if sorted(perm) != list(range(n)):
        raise ValueError("reorder_joints: perm must list every joint once")
    new_link = np.zeros(n + 1, dtype=np.int64)   # old link -> new link
    for k, o in enumerate(perm):
        new_link[o + 1] = k + 1
    parent = np.array([new_link[model["parent"][o]] for o in perm], dtype=np.int32)
    late = [model["names"][perm[k] + 1] for k in range(n) if parent[k] > k]
    if late:
        raise ValueError(f"load_urdf: considered_joints lists {late} before their parent joints; "
                         "list every joint after its parent's (the kernels need parent[j] <= j)")
    out = dict(model)
    out["parent"] = parent
    for key in ("joint_origin", "joint_rot", "joint_axis", "joint_type"):
        if key in model:
            out[key] = np.ascontiguousarray(np.asarray(model[key])[perm])
    links = [0] + [o + 1 for o in perm]
    for key in ("link_mass", "link_com", "link_inertia"):
        out[key] = np.ascontiguousarray(np.asarray(model[key])[links])
    out["frame_link"] = np.asarray([new_link[l] for l in model["frame_link"]], dtype=np.int32)
    out["names"] = [model["names"][0]] + [model["names"][o + 1] for o in perm]
    return out
