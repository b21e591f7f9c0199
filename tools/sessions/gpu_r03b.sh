#!/bin/bash
# Round-3 session-2 A/B: GPU tests, the scan-tree sweep (product vs lib/libblf_v0.so), configs[0],
# and the fbd Euler kernel with the blocked Cholesky against one column per step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
PYTEST_ARGS="-m gpu -x -q --timeout 120 --timeout-method thread tests" bash tools/sessions/gpu_tests.sh || exit 1
for r in 1 2; do
  for v in chol2 chol1; do
    STREAM_TIME=1 BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_$v.so timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
timeout -k 10 200 python bench.py --workload c1 > gpurun_out/bench_c1.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c1.log | cut -c1-400
BATCHES="1 256 1024 2048 4096" bash tools/sessions/gpu_tree_ab.sh > gpurun_out/tree_ab.log 2>&1; cat gpurun_out/tree_ab.log
