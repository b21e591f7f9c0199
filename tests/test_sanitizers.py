"""ASan + UBSan runs of the host code (the stand-in for the reference's Valgrind
memcheck of every unit test, /root/reference/cmake/AddBipedalLocomotionUnitTest.cmake:19-35).

  * the C++17 adapters and their tests (`make -C bipedal-locomotion-framework_amd asan`:
    lib/blf_host_tests_asan, instrumented host code linked to the product lib/libblf.so): the
    host-only cases here, the device-backed cases on a GPU;
  * the CPU oracle (`make -C oracle asan`: liboracle_asan.so) under the oracle's own test files,
    loaded into a child Python with LD_PRELOAD=libasan.so and BLF_ORACLE_LIB.

Every UBSan finding aborts (-fno-sanitize-recover=all); ASan reports abort by default.  Leak
detection stays on for the C++ binary; the Python child runs without it (the interpreter's own
allocations at exit are not ours)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bipedal-locomotion-framework_amd")
ORACLE = os.path.join(ROOT, "oracle")
BIN = os.path.join(PKG, "lib", "blf_host_tests_asan")
ORACLE_ASAN = os.path.join(ORACLE, "liboracle_asan.so")


def _gcc_lib(name):
    return subprocess.check_output(["gcc", f"-print-file-name={name}"], text=True).strip()


@pytest.fixture(scope="module")
def host_asan():
    subprocess.check_call(["make", "-s", "-j8", "-C", PKG, "asan"])
    return BIN


@pytest.fixture(scope="module")
def oracle_asan():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "asan"])
    return ORACLE_ASAN


def _run_host(binary, which, leaks=True):
    env = dict(os.environ, BLF_GOLDEN_DIR=os.path.join(ROOT, "tests", "golden"),
               ASAN_OPTIONS="halt_on_error=1:exitcode=99:detect_leaks=" + ("1" if leaks else "0"),
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([binary, which], capture_output=True, text=True, timeout=900, env=env)
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "runtime error:" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failed" in r.stdout, r.stdout[-2000:]
    return r.stdout


def test_host_adapters_asan_cpu(host_asan):
    out = _run_host(host_asan, "cpu")
    for name in ("ContactList", "ContactPhaseList", "VariablesHandler", "ParametersHandler"):
        assert any(line.startswith(name) and line.rstrip().endswith("ok") for line in out.splitlines()), out


def test_oracle_asan(oracle_asan):
    # the ASan runtime must come first in the preload list; anything already preloaded stays
    preload = " ".join(filter(None, [_gcc_lib("libasan.so"), _gcc_lib("libubsan.so"),
                                     os.environ.get("LD_PRELOAD")]))
    env = dict(os.environ,
               LD_PRELOAD=preload,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               BLF_ORACLE_LIB=oracle_asan)
    files = ["tests/test_oracle.py", "tests/test_oracle_contact.py", "tests/test_oracle_warm.py",
             "tests/test_oracle_phase_expand.py", "tests/test_oracle_closed_loop.py",
             "tests/test_fb_dynamics.py"]
    # the child checks that it really runs the instrumented library
    probe = ("import sys; sys.path.insert(0, 'oracle'); import oracle as O; "
             "assert O.lib()._name.endswith('liboracle_asan.so'), O.lib()._name")
    subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, check=True, timeout=120)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        "-m", "not gpu", *files], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=1200)
    assert "ERROR: AddressSanitizer" not in r.stdout + r.stderr, (r.stdout + r.stderr)[-4000:]
    assert "runtime error:" not in r.stdout + r.stderr, (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
