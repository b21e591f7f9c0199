"""Condense a tools/gpu_stream.sh run (gpurun_out/stream.json + gpurun_out/stream_prof) into
profiles/<tag>_stream_kernels.json: per kernel the event-timed median, the algorithmic bytes and
HBM fraction (tools/stream_bench.py), and the FETCH_SIZE / WRITE_SIZE passes per dispatch
(KiB; FETCH doubled for gfx950's wide coalesced reads, MI355X_MICROARCH.md HBM section), with the
traffic / algorithmic ratio.
  python tools/summarize_stream.py r02 [gpurun_out]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc(path):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(path):
        for r in csv.DictReader(open(f)):
            out[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out")
    lines = [json.loads(l) for l in open(os.path.join(src, "stream.json"))] \
        if open(os.path.join(src, "stream.json")).read().lstrip().startswith("{") else []
    if not lines:
        lines = json.load(open(os.path.join(src, "stream.json")))
    fetch = pmc(os.path.join(src, "stream_prof", "fetch", "*counter_collection.csv"))
    write = pmc(os.path.join(src, "stream_prof", "write", "*counter_collection.csv"))
    counters = {}
    for k in set(fetch) | set(write):
        f = fetch.get(k, {}).get("FETCH_SIZE", [])
        w = write.get(k, {}).get("WRITE_SIZE", [])
        counters[k] = {"dispatches": max(len(f), len(w)),
                       "fetch_x2_corrected_MB": 2 * 1024 * (sum(f) / len(f)) / 1e6 if f else None,
                       "write_MB": 1024 * (sum(w) / len(w)) / 1e6 if w else None}
    bases = collections.Counter(l["kernel"].split("[")[0] for l in lines)
    for l in lines:
        base = l["kernel"].split("[")[0]
        c = counters.get(base)
        # kernels timed in several configurations share one per-dispatch mean: no ratio for them
        if c and c["fetch_x2_corrected_MB"] is not None and c["write_MB"] is not None and bases[base] == 1:
            l["traffic_MB"] = c["fetch_x2_corrected_MB"] + c["write_MB"]
            l["traffic_over_algorithmic"] = l["traffic_MB"] * 1e6 / l["algorithmic_bytes"]
    try:
        build = json.load(open(os.path.join(src, "stream_prof", "build.json")))
    except (OSError, ValueError):
        build = None
    out = {"build": build,
           "source": "tools/gpu_stream.sh: tools/stream_bench.py timed with HIP events (median); "
                     "rocprofv3 --kernel-trace --stats and separate --pmc FETCH_SIZE / WRITE_SIZE "
                     "passes of the same program (per-dispatch means over every dispatch of the "
                     "kernel in the program)",
           "kernels": lines, "pmc_per_kernel": counters}
    dst = os.path.join(ROOT, "profiles", f"{tag}_stream_kernels.json")
    json.dump(out, open(dst, "w"), indent=1)
    for l in lines:
        print(f"{l['kernel']:30s} {l['ms']:.3f} ms  {l['frac']:.3f}  traffic/alg "
              f"{l.get('traffic_over_algorithmic', float('nan')):.2f}")


if __name__ == "__main__":
    main()
