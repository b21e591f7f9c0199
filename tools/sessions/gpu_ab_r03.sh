#!/bin/bash
# Round-3 check on one GPU box: the whole GPU test suite, then event-timed A/B of the streaming /
# dynamics kernels (product library vs the lib/libblf_<name>.so variants in $LIBS), then the SQ
# passes of the kernels in $SQ_KERNELS.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for k in ${TIME_KERNELS:-}; do
  for lib in libblf ${LIBS:-}; do
    BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py $k 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
if [ -n "${SQ_KERNELS:-}" ]; then
  KERNELS="$SQ_KERNELS" SQ_EXTRA=1 timeout -k 10 900 bash tools/gpu_sq.sh > gpurun_out/sq.log 2>&1 || exit 1
fi
echo done
