#!/bin/bash
# Round 4 diagnostics: the c5 loop with the overlap under a kernel trace (per-kernel start / end
# times of a few periods), then the fbd_euler A/B against $FBD_LIBS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04k}
L=$PWD/bipedal-locomotion-framework_amd/lib
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T:-r04k}_trace -o run -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu --c5-overlap 1 > gpurun_out/${T:-r04k}_trace.log 2>&1 || exit 1
f=$(find gpurun_out/${T:-r04k}_trace -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/${T:-r04k}_kernel_trace.csv; wc -l gpurun_out/${T:-r04k}_kernel_trace.csv
for r in 1 2; do
  for lib in libblf ${FBD_LIBS:-}; do
    echo -n "$lib fbd_euler: "
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/${T:-r04k}_fbd_ab.log
