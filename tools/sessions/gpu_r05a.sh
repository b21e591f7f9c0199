#!/bin/bash
# Round 5, first build: the GPU suite, the default bench line, and the bench's kernel trace + PMC
# passes (tools/profile_round.sh).  Each GPU step under its own time limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05a}
timeout -k 10 900 python -u -m pytest tests -v --maxfail=5 -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -2 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench.log | tail -1 | cut -c1-300
timeout -k 10 1500 bash tools/profile_round.sh > gpurun_out/${T}_prof_round.log 2>&1 || { echo "profile_round failed"; tail -5 gpurun_out/${T}_prof_round.log; exit 1; }
echo "profile_round done"
