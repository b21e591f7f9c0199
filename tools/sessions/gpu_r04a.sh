#!/bin/bash
# Round 4, first build: the new c5-window tests first, then the whole GPU suite, the default bench
# line, the c5 line and the QP kernel at 4096 / 65 536; each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T=${TAG:-r04a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5_windows.py -x -v --timeout 240 --timeout-method thread > gpurun_out/${T}_c5win.log 2>&1
rc=$?; tail -8 gpurun_out/${T}_c5win.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -v --maxfail=5 -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -2 gpurun_out/${T}_pytest_gpu.log
# assertion failures (1) still let the benches run; a crash, abort or time limit ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo "bench failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench.log | tail -1 | cut -c1-300
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/${T}_bench_c5.log 2>&1 || { echo "c5 failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench_c5.log | tail -1 | cut -c1-700
{ timeout -k 10 300 python tools/kbench.py && timeout -k 10 300 python tools/kbench.py --batch 65536; } > gpurun_out/${T}_kbench.log 2>&1 || { echo "kbench failed"; exit 1; }
grep -i "ms\|QP/s" gpurun_out/${T}_kbench.log | tail -6
