#!/bin/bash
# Round-3 re-entry check: GPU tests, the headline bench line and a kbench batch sweep,
# each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
for b in 1 1536 4096 16384 65536; do timeout -k 10 120 python tools/kbench.py --reps 20 --batch $b >> gpurun_out/kbench.log 2>&1 || exit 1; done
cat gpurun_out/kbench.log | grep -v amdgpu.ids
echo done
