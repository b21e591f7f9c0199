#!/bin/bash
# Round evidence on one GPU box: gpu tests, the default bench line, then the rocprofv3 passes.
# Every GPU step has its own time limit; anything but a clean pass ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh > gpurun_out/profile.log 2>&1
rc=$?
echo "profile rc=$rc"; tail -3 gpurun_out/profile.log
exit $rc
