#!/bin/bash
# End of round 3: the whole GPU test suite, then the default bench line and the c1 / c5 workload
# lines on the final build, each GPU step under its own time limit (the first failure ends it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-300
for w in c1 c5; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || { echo "$w failed"; exit 1; }
  grep -v amdgpu.ids gpurun_out/bench_$w.log | tail -1 | cut -c1-300
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
