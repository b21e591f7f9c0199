"""CPU tests of bench.py's counter provenance (round-3 verdict item 2): the bench line takes its
counter-derived fields (roofline.traffic, VALU issue, residency) only from a committed profile
summary whose recorded library hash is the hash of the library the process loaded; a newer
summary of another build, or one of another kernel, is skipped, and with no match the fields are
null."""
import json

import pytest

import bench
from blf import native


def _write(root, name, kernel, lib_hash, traffic=1.0e8):
    d = root / "profiles"
    d.mkdir(exist_ok=True)
    s = {"dominant_kernel": kernel, "build": {"lib_src_hash": lib_hash},
         "hbm_traffic_per_launch": {"total_bytes_corrected": traffic}}
    (d / name).write_text(json.dumps(s))


@pytest.fixture
def fake_root(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(native, "build_provenance", lambda: {"lib_src_hash": "aaaa", "matches": True})
    return tmp_path


def test_summary_of_the_loaded_build_is_taken(fake_root):
    _write(fake_root, "r04_v2_summary.json", "dcm_mpc_cold_kernel", "aaaa", traffic=1.1e8)
    _write(fake_root, "r04_v10_summary.json", "dcm_mpc_cold_kernel", "bbbb", traffic=9.9e8)   # newer, other build
    _write(fake_root, "r04_v11_summary.json", "fbd_euler_kernel", "aaaa")                       # other kernel
    s, path = bench.profiled_summary()
    assert path == "profiles/r04_v2_summary.json" and s["build"]["lib_src_hash"] == "aaaa"
    assert bench.profiled_traffic() == (1.1e8, "profiles/r04_v2_summary.json")


def test_newest_matching_summary_wins(fake_root):
    _write(fake_root, "r04_v9_summary.json", "dcm_mpc_cold_kernel", "aaaa", traffic=1.0e8)
    _write(fake_root, "r04_v10_summary.json", "dcm_mpc_cold_kernel", "aaaa", traffic=1.2e8)   # v10 after v9
    assert bench.profiled_traffic() == (1.2e8, "profiles/r04_v10_summary.json")


def test_no_matching_summary_gives_null_fields(fake_root):
    _write(fake_root, "r04_v1_summary.json", "dcm_mpc_cold_kernel", "bbbb")
    assert bench.profiled_summary() == (None, None)
    assert bench.profiled_traffic() == (None, None)
