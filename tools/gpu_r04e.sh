#!/bin/bash
# Round 4 diagnostics: the split QP A/B at large batches, the fbd phase stamps, the c5 per-kernel
# trace.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
for r in 1 2; do
  for B in 65536 16384; do
    for cfg in libblf:0 libblf:1 libblf_search3:1; do
      lib=${cfg%%:*}; sm=${cfg##*:}
      echo -n "$lib split_min=$sm B=$B: "
      BLF_LIB=$L/$lib.so BLF_QP_SPLIT_MIN_BATCH=$sm timeout -k 10 120 python tools/kbench.py --batch $B --reps 20 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done | tee gpurun_out/r04e_split_ab.log
BLF_LIB=$L/libblf_stamps.so timeout -k 10 120 python tools/fbd_stamps.py > gpurun_out/r04e_fbd_stamps.log 2>&1 || { echo "stamps failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/r04e_fbd_stamps.log | tail -14
WORKLOADS=c5 timeout -k 10 300 bash tools/gpu_ktrace_workloads.sh > gpurun_out/r04e_ktrace.log 2>&1 || { echo "ktrace failed"; exit 1; }
tail -12 gpurun_out/r04e_ktrace.log
