#!/bin/bash
# Round 4 re-entry: the default bench line and the c5 line of the round-3 kernels on a fresh box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r04_v0_bench.log 2>&1 || { echo "bench failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_v0_bench.log | tail -1 | cut -c1-400
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/r04_v0_bench_c5.log 2>&1 || { echo "c5 failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_v0_bench_c5.log | tail -1 | cut -c1-600
{ timeout -k 10 300 python tools/kbench.py && timeout -k 10 300 python tools/kbench.py --batch 65536; } > gpurun_out/r04_v0_kbench.log 2>&1 || { echo "kbench failed"; exit 1; }
tail -12 gpurun_out/r04_v0_kbench.log
