#!/bin/bash
# Quintic: GPU kernel tests (bit-exact vs the oracle), then the A/B of the tiled persistent kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -v -x -m gpu -k "quintic or spline" --timeout 120 --timeout-method thread > gpurun_out/r05l_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/r05l_pytest.log | head; tail -1 gpurun_out/r05l_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do STREAM_KERNEL=quintic bash tools/sessions/ab_stream.sh || exit 1; done
