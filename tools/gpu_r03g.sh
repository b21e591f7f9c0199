#!/bin/bash
# Round 3: the hull chain rule (all-triples, registers) against the previous kernel
# (lib/libblf_vhullold.so), 4 alternating rounds of tools/stream_one.py hull; then the wave
# priority diagnostics (lib/libblf_vprio*.so) on kbench; then the hull SQ passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
: > gpurun_out/hull_ab.log
for r in 1 2 3 4; do
  for lib in libblf libblf_vhullold; do
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py hull 2>&1 | grep -v amdgpu.ids >> gpurun_out/hull_ab.log || exit 1
  done
done
cat gpurun_out/hull_ab.log
: > gpurun_out/prio_ab.log
for r in 1 2; do
  for lib in libblf libblf_vprio1 libblf_vprio2; do
    for b in 4096 65536; do
      BLF_LIB=$L/$lib.so timeout -k 10 120 python tools/kbench.py --batch $b --reps 30 2>&1 | grep -v amdgpu.ids >> gpurun_out/prio_ab.log || exit 1
    done
  done
done
cat gpurun_out/prio_ab.log
KERNELS=hull SQ_EXTRA=1 timeout -k 10 600 bash tools/gpu_sq.sh > gpurun_out/sq.log 2>&1 || { tail -5 gpurun_out/sq.log; exit 1; }
echo done
