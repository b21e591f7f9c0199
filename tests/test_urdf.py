"""CPU tests of the URDF loader (blf/urdf.py): the path a user of the reference takes from a robot
description to FloatingBaseDynamicalSystem (iDynTree ModelLoader -> setRobotModel,
FloatingBaseSystemDynamics.cpp:53-74), here to the blf_fb_model layout.  The reference ships no
URDF, so the fixtures are written from the synthetic model (blf/robot.py humanoid24) and read
back: the loaded arrays must equal the model's, and with the soles as massless links on fixed
joints the reduced model must equal the model with sole frames, rigid-body terms included
(oracle/fb_dynamics.py)."""
import numpy as np
import pytest

import fb_dynamics as F
from blf import robot, urdf

MODEL = robot.humanoid24()


def matrix_rpy(R):
    """Roll, pitch, yaw of R = Rz(y) Ry(p) Rx(r) (|p| < pi / 2)."""
    p = np.arcsin(-R[2, 0])
    return np.arctan2(R[2, 1], R[2, 2]), p, np.arctan2(R[1, 0], R[0, 0])


def fmt(v):
    return " ".join(repr(float(x)) for x in v)


def to_urdf(model, soles=False, types=None, extra=""):
    """The model as URDF XML: link l+1 is joint l's child, named after the joint ("<name>_link").
    soles: the sole frames as massless links on fixed joints."""
    names = model["names"]
    lname = lambda l: names[0] if l == 0 else names[l] + "_link"
    out = ['<?xml version="1.0"?>', '<robot name="humanoid24">']
    for l in range(model["n"] + 1):
        I = model["link_inertia"][l]
        out.append(f'  <link name="{lname(l)}"><inertial><origin xyz="{fmt(model["link_com"][l])}" rpy="0 0 0"/>'
                   f'<mass value="{float(model["link_mass"][l])!r}"/>'
                   f'<inertia ixx="{float(I[0, 0])!r}" ixy="{float(I[0, 1])!r}" ixz="{float(I[0, 2])!r}" '
                   f'iyy="{float(I[1, 1])!r}" iyz="{float(I[1, 2])!r}" izz="{float(I[2, 2])!r}"/></inertial></link>')
    for j in range(model["n"]):
        typ = (types or {}).get(names[j + 1], "revolute")
        out.append(f'  <joint name="{names[j + 1]}" type="{typ}"><parent link="{lname(model["parent"][j])}"/>'
                   f'<child link="{lname(j + 1)}"/><origin xyz="{fmt(model["joint_origin"][j])}" '
                   f'rpy="{fmt(matrix_rpy(model["joint_rot"][j]))}"/><axis xyz="{fmt(model["joint_axis"][j])}"/>'
                   f'<limit lower="-3" upper="3" effort="100" velocity="10"/></joint>')
    if soles:
        for f, side in enumerate(("l", "r")):
            out.append(f'  <link name="{side}_sole"/>')
            out.append(f'  <joint name="{side}_sole_fixed" type="fixed"><parent link="{lname(model["frame_link"][f])}"/>'
                       f'<child link="{side}_sole"/><origin xyz="{fmt(model["frame_pose"][f][:3])}" rpy="0 0 0"/></joint>')
    out.append(extra)
    out.append("</robot>")
    return "\n".join(out)


KEYS = ("parent", "joint_origin", "joint_rot", "joint_axis", "link_mass", "link_com", "link_inertia")


def test_urdf_round_trip():
    m = urdf.load_urdf(to_urdf(MODEL))
    assert m["n"] == MODEL["n"] and m["names"] == MODEL["names"]
    for k in KEYS:
        np.testing.assert_allclose(m[k], MODEL[k], rtol=0, atol=1e-15, err_msg=k)
    assert "joint_type" not in m and len(m["frame_link"]) == 0


def test_urdf_sole_frames_on_fixed_joints():
    """Massless sole links on fixed joints, exposed as frames: the reduced model is the model with
    sole frames, and its mass matrix, bias forces and sole Jacobians agree with it."""
    m = urdf.load_urdf(to_urdf(MODEL, soles=True), frames=("l_sole", "r_sole"))
    assert m["n"] == MODEL["n"] and m["names"] == MODEL["names"]
    np.testing.assert_array_equal(m["frame_link"], MODEL["frame_link"])
    np.testing.assert_allclose(m["frame_pose"], MODEL["frame_pose"], atol=1e-15)
    for k in KEYS:
        np.testing.assert_allclose(m[k], MODEL[k], rtol=0, atol=1e-15, err_msg=k)
    st = robot.random_states(MODEL, 1, seed=7)
    st = {k: v[0] for k, v in st.items()}
    K = F.kinematics(MODEL, st["base_pos"], st["base_rot"], st["joint_pos"], st["base_vel"], st["joint_vel"])
    Km = F.kinematics(m, st["base_pos"], st["base_rot"], st["joint_pos"], st["base_vel"], st["joint_vel"])
    M, h = F.mass_and_bias(MODEL, K)
    Mm, hm = F.mass_and_bias(m, Km)
    np.testing.assert_allclose(Mm, M, rtol=1e-13, atol=1e-13 * np.abs(M).max())
    np.testing.assert_allclose(hm, h, rtol=1e-13, atol=1e-13 * np.abs(h).max())
    for f in range(2):
        np.testing.assert_allclose(F.frame_state(m, Km, f)[3], F.frame_state(MODEL, K, f)[3], atol=1e-13)


def test_urdf_joint_types_and_considered_joints():
    """continuous = revolute, prismatic kept as such; joints outside considered_joints are locked
    (merged), as iDynTree's reduced loader does -- the same model as reduce_fixed_joints."""
    types = {"neck_pitch": "continuous", "torso_roll": "prismatic"}
    m = urdf.load_urdf(to_urdf(MODEL, types=types))
    ref = robot.with_joint_types(MODEL, prismatic=("torso_roll",))
    np.testing.assert_array_equal(m["joint_type"], ref["joint_type"])
    keep = [nm for nm in MODEL["names"][1:] if nm not in ("l_elbow", "r_elbow", "neck_pitch")]
    mr = urdf.load_urdf(to_urdf(MODEL), considered_joints=keep)
    red = robot.reduce_fixed_joints(MODEL, ("l_elbow", "r_elbow", "neck_pitch"))
    assert mr["names"] == red["names"]
    for k in KEYS:
        np.testing.assert_allclose(mr[k], red[k], rtol=0, atol=1e-14, err_msg=k)


def test_urdf_dfs_order():
    """Joints in depth-first preorder whatever the document order: parent[j] <= j and every subtree
    a contiguous run (the dynamics kernel's prefix-sum subtree sums rely on it)."""
    text = to_urdf(MODEL)
    lines = text.split("\n")
    joints = [ln for ln in lines if ln.lstrip().startswith("<joint")]
    rest = [ln for ln in lines if not ln.lstrip().startswith("<joint") and ln != "</robot>"]
    m = urdf.load_urdf("\n".join(rest + joints[::-1] + ["</robot>"]))
    n, parent = m["n"], m["parent"]
    assert all(0 <= parent[j] <= j for j in range(n))
    anc = [set() for _ in range(n)]
    for j in range(n):
        p = parent[j]
        anc[j] = ({p - 1} | anc[p - 1]) if p > 0 else set()
    for j in range(n):
        members = [k for k in range(n) if k == j or j in anc[k]]
        assert members == list(range(j, j + len(members)))
    assert sorted(m["names"]) == sorted(MODEL["names"])


@pytest.mark.parametrize("bad,msg", [
    ('<joint name="x" type="floating"><parent link="base"/><child link="extra"/></joint><link name="extra"/>',
     "not supported"),
    ('<link name="orphan"/>', "trees"),
    ('<joint name="y" type="revolute"><parent link="base"/><child link="l_hip_yaw_link"/></joint>', "two joints"),
])
def test_urdf_errors(bad, msg):
    with pytest.raises(ValueError, match=msg):
        urdf.load_urdf(to_urdf(MODEL, extra=bad))
    with pytest.raises(ValueError, match="not a link"):
        urdf.load_urdf(to_urdf(MODEL), frames=("nope",))


def test_urdf_considered_joints_order():
    """The degrees of freedom follow considered_joints' order (iDynTree's reduced loader), here the
    right leg's chain before the left's: the rigid-body terms are the depth-first model's with q,
    qdot, tau and M permuted the same way; a list that names a joint before its parent's is
    refused."""
    names = MODEL["names"][1:]
    left = [nm for nm in names if nm.startswith("l_")]
    right = [nm for nm in names if nm.startswith("r_")]
    rest = [nm for nm in names if nm not in left and nm not in right]
    order = rest + right + left
    m = urdf.load_urdf(to_urdf(MODEL), considered_joints=order)
    assert m["names"][1:] == order
    n = MODEL["n"]
    perm = [names.index(nm) for nm in order]
    assert all(0 <= m["parent"][j] <= j for j in range(n))
    st = robot.random_states(MODEL, 1, seed=5)
    K = F.kinematics(MODEL, st["base_pos"][0], st["base_rot"][0], st["joint_pos"][0], st["base_vel"][0],
                     st["joint_vel"][0])
    M0, h0 = F.mass_and_bias(MODEL, K)
    Kp = F.kinematics(m, st["base_pos"][0], st["base_rot"][0], st["joint_pos"][0][perm], st["base_vel"][0],
                      st["joint_vel"][0][perm])
    M1, h1 = F.mass_and_bias(m, Kp)
    rows = list(range(6)) + [6 + j for j in perm]
    np.testing.assert_allclose(M1, M0[np.ix_(rows, rows)], rtol=0, atol=1e-12)
    np.testing.assert_allclose(h1, h0[rows], rtol=0, atol=1e-11)
    child_first = [nm for nm in order if nm != "l_knee"] + ["l_knee"]
    child_first.insert(child_first.index([nm for nm in left if nm != "l_knee"][0]), "l_knee")
    with pytest.raises(ValueError, match="before their parent"):
        urdf.load_urdf(to_urdf(MODEL), considered_joints=child_first)


# ---- the C++ adapter's loader (host/src/UrdfLoader.cpp) against this one ------------------------
import json
import os
import subprocess

_PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bipedal-locomotion-framework_amd")
_BIN = os.path.join(_PKG, "lib", "blf_host_tests")


def _cpp_load(tmp_path, text, frames=(), considered=None, base=None):
    if not os.path.exists(_BIN):
        subprocess.check_call(["make", "-s", "-j8", "-C", _PKG])
    path = tmp_path / "robot.urdf"
    path.write_text(text)
    args = [_BIN, "urdf", str(path), ",".join(frames) or "-",
            "*" if considered is None else (",".join(considered) or "-"), base or "-"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=60)
    out = json.loads(r.stdout)
    assert (r.returncode == 0) == ("error" not in out), r.stdout + r.stderr
    return out


def _reversed_joints(text):
    lines = text.split("\n")
    joints = [ln for ln in lines if ln.lstrip().startswith("<joint")]
    rest = [ln for ln in lines if not ln.lstrip().startswith("<joint") and ln != "</robot>"]
    return "\n".join(rest + joints[::-1] + ["</robot>"])


_ORDER = ([nm for nm in MODEL["names"][1:] if not nm.startswith(("l_", "r_"))]
          + [nm for nm in MODEL["names"][1:] if nm.startswith("r_")]
          + [nm for nm in MODEL["names"][1:] if nm.startswith("l_")])
_CASES = {
    "plain": (to_urdf(MODEL), {}),
    "soles": (to_urdf(MODEL, soles=True), dict(frames=("l_sole", "r_sole"))),
    "types": (to_urdf(MODEL, types={"neck_pitch": "continuous", "torso_roll": "prismatic"}), {}),
    "locked": (to_urdf(MODEL, soles=True), dict(frames=("r_sole",), considered_joints=[
        nm for nm in MODEL["names"][1:] if nm not in ("l_elbow", "r_elbow", "neck_pitch")])),
    "order": (to_urdf(MODEL), dict(considered_joints=_ORDER)),
    "document order": (_reversed_joints(to_urdf(MODEL)), {}),
    "xml features": (to_urdf(MODEL).replace('<?xml version="1.0"?>', '<?xml version="1.0"?>\n<!DOCTYPE robot>\n'
                                              '<!-- a comment with <tags> -->').replace(
        '<robot name="humanoid24">', "<robot name='humanoid&amp;24'>\n<material name=\"grey\"><color rgba=\"0.5 0.5 0.5 1\"/></material>"), {}),
}


@pytest.mark.parametrize("case", list(_CASES))
def test_cpp_urdf_loader_matches_python(tmp_path, case):
    """blf::loadUrdf (the C++ adapter's setRobotModel input) gives the Python loader's model: the
    same DoF names and order, parents, frames and types bit for bit, the floating-point arrays to
    1e-15 (the 3 x 3 products may round differently)."""
    text, kw = _CASES[case]
    py = urdf.load_urdf(text, **kw)
    cpp = _cpp_load(tmp_path, text, frames=kw.get("frames", ()), considered=kw.get("considered_joints"))
    n = py["n"]
    assert cpp["n"] == n and cpp["names"] == py["names"][1:]
    np.testing.assert_array_equal(cpp["parent"], py["parent"])
    np.testing.assert_array_equal(cpp["joint_type"], py.get("joint_type", np.zeros(n, dtype=np.int32)))
    np.testing.assert_array_equal(cpp["frame_link"], py["frame_link"])
    for k in ("joint_origin", "joint_rot", "joint_axis", "link_mass", "link_com", "link_inertia", "frame_pose"):
        np.testing.assert_allclose(np.reshape(cpp[k], np.shape(py[k])), py[k], rtol=0, atol=1e-15, err_msg=k)


@pytest.mark.parametrize("bad", [
    '<joint name="x" type="floating"><parent link="base"/><child link="extra"/></joint><link name="extra"/>',
    '<link name="orphan"/>',
    '<joint name="y" type="revolute"><parent link="base"/><child link="l_hip_yaw_link"/></joint>',
    '<link name="base"/>',
    '<joint name="z" type="revolute"><parent link="base"/><child link="nowhere"/></joint>',
    '<link name="bad"><inertial><mass value="-1"/></inertial></link><joint name="w" type="fixed">'
    '<parent link="base"/><child link="bad"/></joint>',
])
def test_cpp_urdf_loader_refuses(tmp_path, bad):
    """Both loaders refuse the same malformed models."""
    text = to_urdf(MODEL, extra=bad)
    with pytest.raises(ValueError):
        urdf.load_urdf(text)
    assert "error" in _cpp_load(tmp_path, text)
    assert "error" in _cpp_load(tmp_path, to_urdf(MODEL), frames=("nope",))
    assert "error" in _cpp_load(tmp_path, to_urdf(MODEL), considered=["no_such_joint"])
    assert "error" in _cpp_load(tmp_path, "<robot><link name='a'></robot>")   # malformed XML
    child_first = [nm for nm in _ORDER if nm != "l_knee"]
    child_first.insert(child_first.index("l_hip_pitch") if "l_hip_pitch" in child_first else 0, "l_knee")
    with pytest.raises(ValueError):
        urdf.load_urdf(to_urdf(MODEL), considered_joints=child_first)
    assert "before their parent" in _cpp_load(tmp_path, to_urdf(MODEL), considered=child_first)["error"]
