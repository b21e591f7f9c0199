#!/bin/bash
# The bench's other workloads (configs[0] c1, closed loop c3/c5, receding horizon rh) and the
# batch-scaling kbench, each under its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for w in c1 c3 c5 rh; do
    timeout -k 10 300 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || { echo "$w failed"; exit 1; }
    echo "$w:"; grep -v amdgpu.ids gpurun_out/bench_$w.log | tail -1 | cut -c1-400
done
: > gpurun_out/kb_scale.log
for b in 1536 4096 16384 65536; do
    timeout -k 10 120 python tools/kbench.py --reps 20 --batch $b 2>&1 | grep -v amdgpu.ids >> gpurun_out/kb_scale.log || { echo "kbench $b failed"; exit 1; }
done
cat gpurun_out/kb_scale.log
