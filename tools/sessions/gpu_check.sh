#!/bin/bash
# One GPU session: gpu tests, then a short bench.  Each GPU step has its own time limit; a
# fault / abort / timeout (anything but pass or test-failure) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -q"}
timeout -k 10 480 python -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
BENCH_ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 3}
timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -5 gpurun_out/bench.log
exit $rc2
