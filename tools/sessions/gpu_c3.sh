#!/bin/bash
# configs[0] / configs[2] lines and the kernel-trace stats of the configs[2] pipeline step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in c1 c3; do
    timeout -k 10 300 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/bench_$w.log; exit 1; }
    echo "$w:"; grep -v amdgpu.ids gpurun_out/bench_$w.log | tail -1 | cut -c1-600
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/c3prof -o run -- python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu > gpurun_out/c3prof.log 2>&1 || { echo "c3 prof failed"; exit 1; }
cat gpurun_out/c3prof/run_kernel_stats.csv | cut -d, -f1-4 | head -20
