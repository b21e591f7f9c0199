#!/bin/bash
# Round 3, last: the iterative-ILP scheduler on the remaining kernel TUs (lib/libblf_vall.so)
# against the product: streaming kernels (tools/stream_one.py) and the IPM kernel (kbench at
# N = 150, the interior point path), two alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
: > gpurun_out/sched_rest_ab.log
for r in 1 2; do
  for lib in libblf libblf_vall; do
    for k in rollout hull quintic contact fbk fbk_euler; do
      BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py $k 2>&1 | grep -v amdgpu.ids >> gpurun_out/sched_rest_ab.log || exit 1
    done
    BLF_LIB=$L/$lib.so timeout -k 10 120 python tools/kbench.py --batch 4096 --horizon 150 --reps 10 2>&1 | grep -v amdgpu.ids >> gpurun_out/sched_rest_ab.log || exit 1
  done
done
cat gpurun_out/sched_rest_ab.log
