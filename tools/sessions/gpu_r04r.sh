#!/bin/bash
# Round 4: event-timed A/B of the streaming kernels (hull, quintic) against variant libraries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
for r in 1 2; do
  for k in ${KS:-hull quintic}; do
    for lib in libblf ${LIBS:-}; do
      echo -n "$lib: "
      BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py $k 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done | tee gpurun_out/${TAG:-r04r}_stream_ab.log
