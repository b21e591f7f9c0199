"""Median per-dispatch SQ counters from gpurun_out/sq/<target><n>/ (tools/gpu_sq.sh).
  python tools/sq_summary.py <target> <kernel-name-prefix>"""
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
