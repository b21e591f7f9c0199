#!/bin/bash
# GPU test run only (PYTEST_ARGS overrides the selection).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${PYTEST_ARGS:-tests -m gpu -q -x} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
exit $rc
