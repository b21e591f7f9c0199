"""Condense a tools/profile_round.sh run (gpurun_out/prof) into profiles/<tag>_*.

Writes <tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary, verbatim) and
<tag>_summary.json: per-dispatch averages of the PMC counters for every kernel, and for the
dominant kernel the HBM traffic per launch computed as the guide prescribes
(MI355X_MICROARCH.md 'HBM'): FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE under-reports
wide coalesced reads by 2x on gfx950, so both the raw and the x2-corrected read bytes are given.
  python tools/summarize_profile.py r01 [gpurun_out/prof]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def occupancy(d, avg_ns):
    """Achieved residency of the dominant kernel: SQ_WAVE_CYCLES (counted in units of 4 cycles on
    gfx9) over the chip's SIMD cycles in the kernel time, i.e. waves resident per SIMD on
    average, next to the compile-time limit (tools/kernel_resources)."""
    wc = d.get("SQ_WAVE_CYCLES", {}).get("mean_per_dispatch")
    if wc is None:
        return None
    return {"waves_per_simd_achieved": 4.0 * wc / (SIMDS * CLOCK_HZ * avg_ns * 1e-9),
            "note": "SQ_WAVE_CYCLES x 4 / (1024 SIMDs x 2.4 GHz x kernel time); the tail of the "
                    "last round of workgroups lowers the average"}


def resources():
    """Compile-time VGPRs / spills / occupancy of the QP kernels (hipcc -Rpass-analysis)."""
    import re
    import subprocess
    src = os.path.join(ROOT, "bipedal-locomotion-framework_amd", "csrc", "dcm_mpc_as.hip")
    try:
        out = subprocess.run(
            ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
             "-ffp-contract=off", "-I" + os.path.join(ROOT, "include"),
             "-I" + os.path.dirname(src), "-c", src, "-o", os.devnull, "--cuda-device-only",
             "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=600).stderr
    except (OSError, subprocess.SubprocessError):
        return None
    res, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            key = {"VGPRs Spill": "vgpr_spill", "ScratchSize [bytes/lane]": "scratch_bytes_per_lane",
                   "Occupancy [waves/SIMD]": "occupancy_waves_per_simd",
                   "LDS Size [bytes/block]": "static_lds_bytes"}.get(m.group(1), m.group(1).lower())
            res[cur][key] = int(m.group(2))
    # the instances the bench runs: cold <KPL 2, no lambda out, per-knot input, kTreePad> (c2) and
    # warm <KPL 2, lambda out, phase-indexed input, kTreePad> (rh)
    keep = {k: v for k, v in res.items() if "dcm_mpc_cold_kernelILi2ELb0ELb0ELi1E" in k
            or "dcm_mpc_warm_kernelILi2ELb1ELb1ELi1E" in k}
    return {("dcm_mpc_cold_kernel<2> (c2)" if "cold" in k else "dcm_mpc_warm_kernel<2> (rh)"): v
            for k, v in keep.items()}


def counters(path):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        out[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


SIMDS = 1024          # 256 CUs x 4 SIMDs
CLOCK_HZ = 2.4e9      # peak engine clock


def valu_issue(d, avg_ns):
    """The roof that binds the QP kernel: VALU issue.  SQ_INSTS_VALU counts wave-instructions per
    dispatch; an fp64 FMA / MUL / ADD takes 4 SIMD cycles (16 lanes per cycle), every other VALU
    instruction 2 (SIMD-32); the chip offers SIMDS x clock x time SIMD cycles."""
    n = d.get("SQ_INSTS_VALU", {}).get("mean_per_dispatch")
    if n is None:
        return None
    f64 = [d.get(c, {}).get("mean_per_dispatch") for c in
           ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64")]
    n64 = sum(f64) if None not in f64 else n
    cycles = 4 * n64 + 2 * (n - n64)
    out = {"valu_insts_per_launch": n,
           "valu_cycles_per_launch": cycles,
           "chip_simd_cycles_per_launch": SIMDS * CLOCK_HZ * avg_ns * 1e-9,
           "frac": cycles / (SIMDS * CLOCK_HZ * avg_ns * 1e-9)}
    if None not in f64:
        out["fp64_insts_per_launch"] = {"fma": f64[0], "mul": f64[1], "add": f64[2]}
    return out


def stall_breakdown(d):
    """Where a wave's cycles go (SQ counters in quad-cycles; WAIT_ANY + WAIT_INST_ANY +
    ACTIVE_INST_ANY = WAVE_CYCLES, MI355X_MICROARCH.md counter table): parked on s_waitcnt /
    barriers, issue-stalled on dependencies, issuing (of which VALU, LDS, scalar)."""
    g = lambda c: d.get(c, {}).get("mean_per_dispatch")
    w, waves = g("SQ_WAVE_CYCLES"), g("SQ_WAVES")
    parts = {"wait_any": g("SQ_WAIT_ANY"), "wait_inst_any": g("SQ_WAIT_INST_ANY"),
             "active_inst_any": g("SQ_ACTIVE_INST_ANY"), "active_inst_valu": g("SQ_ACTIVE_INST_VALU"),
             "active_inst_lds": g("SQ_ACTIVE_INST_LDS"), "active_inst_sca": g("SQ_ACTIVE_INST_SCA"),
             "wait_inst_lds": g("SQ_WAIT_INST_LDS"), "lds_bank_conflict": g("SQ_LDS_BANK_CONFLICT")}
    if not w or not waves or parts["wait_any"] is None:
        return None
    return {"wave_cycles_per_wave": 4.0 * w / waves,
            "frac_of_wave_cycles": {k: (v / w if v is not None else None) for k, v in parts.items()},
            "per_wave_cycles": {k: (4.0 * v / waves if v is not None else None) for k, v in parts.items()},
            "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; per-wave cycles = 4 x count / SQ_WAVES"}


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "prof")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
    pmc = collections.defaultdict(dict)
    for sub in ("fetch", "write", "sq", "sq2", "sq3"):
        for kname, cs in counters(os.path.join(src, sub, "run_counter_collection.csv")).items():
            for c, v in cs.items():
                pmc[kname][c] = {"dispatches": len(v), "mean_per_dispatch": sum(v) / len(v)}
    dom = max(stats, key=lambda k: float(stats[k]["TotalDurationNs"]))
    d = pmc.get(dom, {})
    fetch_kib = d.get("FETCH_SIZE", {}).get("mean_per_dispatch")
    write_kib = d.get("WRITE_SIZE", {}).get("mean_per_dispatch")
    try:
        build = json.load(open(os.path.join(src, "build.json")))
    except (OSError, ValueError):
        build = None
    summary = {
        # the library these counters come from (blf/native.py build_provenance on the box):
        # bench.py uses a summary only when its lib_src_hash is the measured library's
        "build": build,
        "source": "tools/profile_round.sh (rocprofv3 --kernel-trace --stats; separate --pmc passes "
                  "FETCH_SIZE | WRITE_SIZE | SQ_*) on `python3 bench.py --steps 10 --warmup 2 --no-cpu`",
        "dominant_kernel": dom,
        "dominant_avg_ns": float(stats[dom]["AverageNs"]),
        "dominant_calls": int(stats[dom]["Calls"]),
        "hbm_traffic_per_launch": None if fetch_kib is None or write_kib is None else {
            "fetch_bytes_raw": fetch_kib * 1024,
            "fetch_bytes_x2_corrected": 2 * fetch_kib * 1024,
            "write_bytes": write_kib * 1024,
            "total_bytes_corrected": (2 * fetch_kib + write_kib) * 1024,
            "note": "FETCH_SIZE/WRITE_SIZE are KiB and count L2 misses to the fabric "
                    "(Infinity-Cache hits included); gfx950 FETCH_SIZE reads 1/2 of wide "
                    "coalesced stream bytes (MI355X_MICROARCH.md HBM section)"},
        "valu_issue": valu_issue(d, float(stats[dom]["AverageNs"])),
        "stall_breakdown": stall_breakdown(d),
        "occupancy": occupancy(d, float(stats[dom]["AverageNs"])),
        "kernel_resources": resources(),
        # dynamic LDS of the dominant kernel at the bench's configs[1] (dcm_mpc_as.hip launch_kpl:
        # fp64 facet rows [M][S] double2 + [M][S] double, S = 2 ceil(N / 2), N = 100, M = 8)
        "lds_bytes_per_qp": 3 * 8 * 8 * 100,
        "qps_per_cu_by_lds": (160 * 1024) // (3 * 8 * 8 * 100),
        "kernel_avg_ns": {k: float(v["AverageNs"]) for k, v in stats.items()},
        "pmc_per_kernel": pmc,
    }
    with open(os.path.join(dst, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: summary[k] for k in ("dominant_kernel", "dominant_avg_ns",
                                               "hbm_traffic_per_launch")}, indent=1))


if __name__ == "__main__":
    main()
