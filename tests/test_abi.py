"""CPU tests of the drop-in boundary: the library loads, exports every entry point the header
declares, and its host-only entry points behave (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import pytest

from blf import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "blf", "blf_c.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(blf_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_and_library_exports_every_symbol():
    declared = _declared()
    assert set(declared) == set(native.EXPORTED), (declared, native.EXPORTED)
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (blf_[a-z0-9_]+)$", out, flags=re.M))
    missing = set(declared) - exported
    assert not missing, missing
    # the round-4 paths measured slower and never the default (split search / certify kernels,
    # the closed loop's begin / finish overlap with its masked kernels and CU-ranged streams)
    # are gone from the product
    assert not set(native.REMOVED) & exported, set(native.REMOVED) & exported
    assert not set(native.REMOVED) & set(declared)


def test_library_was_built_from_this_tree():
    """Build provenance: the source hash compiled into blf_version() (Makefile SRC_HASH) equals the
    hash of the kernel / C-ABI sources in this tree, so the loaded .so is the committed code."""
    prov = native.build_provenance()
    assert prov["tree_src_hash"] is not None
    assert prov["matches"], prov


def test_library_is_built_for_gfx950_only():
    # the .hip_fatbin bundle names one code object per offload target
    out = subprocess.run(["strings", native.LIB_PATH], capture_output=True, text=True).stdout
    targets = set(re.findall(r"amdgcn-amd-amdhsa--(gfx\w+)", out))
    assert targets == {"gfx950"}, targets
    assert "nvptx" not in out


def test_host_only_entry_points_without_gpu():
    L = native.lib()
    p = native.default_params(100)
    assert p.horizon == 100 and p.max_facets == 8 and p.max_iter == 50
    assert p.tol_mu == 1e-16 and p.tol_primal == 1e-10 and p.tol_dual == 1e-9
    assert tuple(p.w_xi) == (100.0, 100.0) and tuple(p.w_terminal) == (1000.0, 1000.0)
    assert native.flops_per_iter(100, 500) == 149 * 500 + 255 * 100
    assert native.version().startswith("blf-mi355x")
    # argument validation happens before any device work: a null handle is rejected
    rc = L.blf_dcm_mpc_solve(None, ctypes.byref(p), None, 1, None, None)
    assert rc == 1 and "null" in native.last_error()
    rc = L.blf_lti_euler_integrate(None, 2, 1, None, None, 1, None, None, 1, 0.0, 1.0, 0.1, None)
    assert rc == 1


def test_create_fails_loudly_without_a_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    with pytest.raises(native.BlfError) as e:
        native.Handle(0)
    assert e.value.code == 2


def test_oracle_is_not_linked_by_the_product():
    for lib in ("libblf.so", "libblf_host.so"):
        path = os.path.join(os.path.dirname(native.LIB_PATH), lib)
        out = subprocess.run(["ldd", path], capture_output=True, text=True).stdout
        assert "oracle" not in out
        syms = subprocess.run(["nm", "-D", path], capture_output=True, text=True).stdout
        assert "orc_" not in syms


def test_lib_loads_after_torch_runtime():
    """native.lib() maps torch's HIP runtime before libblf.so, so the library binds to it (one
    runtime per process; loaded first, it would own the device and torch would see none)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'bipedal-locomotion-framework_amd'); "
            "from blf import native; native.lib(); assert 'torch' in sys.modules")
    subprocess.check_call([sys.executable, "-c", code], cwd=ROOT)


def test_reserved_fields_must_be_zero():
    """blf_posture_law.reserved and blf_joint_impedance.reserved are checked like the QP structs'
    (argument validation before any device work; the handle is only compared with null there)."""
    L = native.lib()
    fake_handle = ctypes.c_void_p(1)
    law = native.PostureLaw()
    law.ndof, law.reserved = 3, 1
    rc = L.blf_dcm_posture_reference(fake_handle, ctypes.byref(law), None, None, 2, 0, None, None)
    assert rc == 1 and "reserved" in native.last_error()
    imp = native.JointImpedance()
    imp.ndof, imp.reserved = 3, 7
    rc = L.blf_fbd_euler_integrate_impedance(None, None, None, ctypes.byref(imp), None, None, 0,
                                             0.0, 1.0, 0.1, None)
    assert rc == 1 and "reserved" in native.last_error()
