#!/bin/bash
# Round-3 evidence run 1 of 2: GPU tests, the default bench line, the workloads (c1 c3 c5 rh) and
# the batch-scaling kbench, then the configs[0] per-phase stamps (stamp build, B = 1, N = 50).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
PYTEST_ARGS="-m gpu -x -q --timeout 120 --timeout-method thread tests" bash tools/sessions/gpu_tests.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-300
bash tools/sessions/gpu_workloads.sh || exit 1
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_stamps.so timeout -k 10 100 python tools/kbench.py --reps 20 --batch 1 --horizon 50 > gpurun_out/stamps_c1.log 2>&1 || exit 1
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_stamps.so timeout -k 10 100 python tools/kbench.py --reps 10 --batch 4096 > gpurun_out/stamps_c2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamps_c1.log | tail -30
echo done
