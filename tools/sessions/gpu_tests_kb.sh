#!/bin/bash
# GPU test suite, then the kernel micro-benchmark (tools/kbench.py) of the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${PYTEST_ARGS:-tests -m gpu -q -x} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/kbench.py --reps 20 > gpurun_out/kb.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/kb.log | tail -2
