#!/bin/bash
# Scan-tree A/B: kbench over batch sizes for the product library and lib/libblf_v0.so (the
# previous build), N = 100 and N = 50.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for N in 100 50; do
  for b in ${BATCHES:-1 64 256 1024 2048 4096}; do
    for lib in libblf.so libblf_v0.so; do
      BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$lib timeout -k 10 100 python tools/kbench.py --reps 50 --batch $b --horizon $N 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
