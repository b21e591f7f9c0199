#!/bin/bash
# Round 3: the hull chain rule (all-triples, registers) against the previous kernel
# (lib/libblf_vhullr1.so: the first all-triples build; lib/libblf_vhullold.so: Andrew's chain), 4
# alternating rounds of tools/stream_one.py hull after the hull parity tests; then the hull SQ passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_staging.py tests/test_gpu_kernels.py -q -x -m gpu > gpurun_out/pytest_hull.log 2>&1 || { tail -20 gpurun_out/pytest_hull.log; exit 1; }
tail -2 gpurun_out/pytest_hull.log
: > gpurun_out/hull_ab.log
for r in 1 2 3 4; do
  for lib in libblf libblf_vhullr1 libblf_vhullold; do
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py hull 2>&1 | grep -v amdgpu.ids >> gpurun_out/hull_ab.log || exit 1
  done
done
cat gpurun_out/hull_ab.log
KERNELS=hull SQ_EXTRA=1 timeout -k 10 600 bash tools/gpu_sq.sh > gpurun_out/sq.log 2>&1 || { tail -5 gpurun_out/sq.log; exit 1; }
echo done
