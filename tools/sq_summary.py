"""Median per-dispatch SQ counters from gpurun_out/sq/<target><n>/ (tools/gpu_sq.sh).
  python tools/sq_summary.py <target> <kernel-name-prefix> [out.json]"""
import collections
import csv
import glob
import sys

target, prefix = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(list)
for d in sorted(glob.glob(f"gpurun_out/sq/{target}[0-9]*/")):
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if r["Kernel_Name"].startswith(prefix):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
med = {c: sorted(v)[len(v) // 2] for c, v in vals.items()}
w = med.get("SQ_WAVES", 1.0)
for c in sorted(med):
    print(f"{c:28s} {med[c]:16.0f}   per wave {med[c] / w:12.1f}")
if len(sys.argv) > 3:
    import json
    wc = med.get("SQ_WAVE_CYCLES")
    out = {"source": f"tools/gpu_sq.sh target {target}, kernel {prefix}: median per dispatch over "
                     f"the rocprofv3 --pmc passes (gpurun_out/sq/{target}N)",
           "median_per_dispatch": med,
           "per_wave": {c: v / w for c, v in med.items()},
           "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* / SQ_LDS_BANK_CONFLICT count quad-cycles"}
    if wc:
        out["frac_of_wave_cycles"] = {c: med[c] / wc for c in med
                                      if c.startswith(("SQ_WAIT", "SQ_ACTIVE_INST", "SQ_LDS_BANK"))}
    import os
    bj = "gpurun_out/sq/build.json"   # the library the passes ran (tools/gpu_sq.sh writes it)
    if os.path.exists(bj):
        out["build"] = json.load(open(bj))
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1)
