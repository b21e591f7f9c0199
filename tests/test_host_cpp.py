"""Runs the C++17 adapter tests (bipedal-locomotion-framework_amd/host/tests/host_tests.cpp):
the reference's Catch2 tests for ContactList, ContactPhaseList and VariablesHandler on the host,
and the device-backed IntegratorTest / ConvexHullHelper / QuinticSpline / planner /
ContinousContactModelTest / FloatingBaseSystemKinematics cases."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bipedal-locomotion-framework_amd")
BIN = os.path.join(PKG, "lib", "blf_host_tests")


def _ensure_built():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG])


def _run(which):
    _ensure_built()
    env = dict(os.environ, BLF_GOLDEN_DIR=os.path.join(ROOT, "tests", "golden"))
    r = subprocess.run([BIN, which], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout, r.stdout
    return r.stdout


def test_host_bookkeeping_tests():
    out = _run("cpu")
    for name in ("ContactList", "ContactPhaseList", "VariablesHandler", "ParametersHandler",
                 "Integrator - host-side system"):
        assert any(line.startswith(name) and line.rstrip().endswith("ok") for line in out.splitlines())


@pytest.mark.gpu
def test_host_device_tests():
    out = _run("gpu")
    for name in ("Integrator - Linear system", "Convex Hull helper (2-D)",
                 "Convex Hull helper (3-D, ConvexHullHelperTest.cpp)", "QuinticSpline",
                 "TimeVaryingDCMPlanner advance", "Continuous Contact",
                 "FloatingBaseSystemKinematics", "FloatingBaseDynamicalSystem",
                 "Integrator - host-side system == device LTI", "Integrator - LTI of any size",
                 "Convex Hull helper (n-D)"):
        assert any(line.startswith(name) and line.rstrip().endswith("ok") for line in out.splitlines()), out
