#!/bin/bash
# Round 5: the stage-2 list path first (the tests that hand QPs over), then the whole GPU suite,
# the default bench line and the bench's kernel trace + PMC passes.  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5_windows.py tests/test_gpu_dcm_mpc.py -v -x -m gpu --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest_stage2.log 2>&1
rc=$?; grep -E "FAILED|ERROR|Error" gpurun_out/${T}_pytest_stage2.log | head -5; tail -1 gpurun_out/${T}_pytest_stage2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench.log | tail -1 | cut -c1-300
[ "${PROF:-1}" = 1 ] || exit 0
timeout -k 10 1500 bash tools/profile_round.sh > gpurun_out/${T}_prof_round.log 2>&1 || { echo "profile_round failed"; tail -5 gpurun_out/${T}_prof_round.log; exit 1; }
echo "profile_round done"
