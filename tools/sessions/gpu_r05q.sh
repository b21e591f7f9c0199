#!/bin/bash
# The closed loop's cold-after-hand-over rule: closed-loop / c5-window GPU tests, the c5 bench twice
# and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_closed_loop.py tests/test_gpu_c5_windows.py -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -20; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/${T}_c5_$r.log 2>&1 || { echo "c5 failed"; tail -3 gpurun_out/${T}_c5_$r.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_c5_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
done
WORKLOADS=c5 bash tools/gpu_ktrace_workloads.sh
