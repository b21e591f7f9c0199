#!/bin/bash
# Round 5: the whole GPU suite, then every workload's bench line (c2 default, c1, c3, rh, mc, c5 at
# two and one stream groups).  Each GPU step under its own time limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05g}
timeout -k 10 900 python -u -m pytest tests -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for w in c2 c1 c3 rh mc; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/${T}_bench_$w.log 2>&1 || { echo "bench $w failed"; tail -3 gpurun_out/${T}_bench_$w.log; exit 1; }
  echo -n "$w: "; grep -v amdgpu.ids gpurun_out/${T}_bench_$w.log | tail -1 | cut -c1-220
done
for g in 2 1; do
  timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/${T}_c5_g$g.log 2>&1 || { echo "c5 g=$g failed"; tail -3 gpurun_out/${T}_c5_g$g.log; exit 1; }
  echo -n "c5 groups=$g: "; grep -v amdgpu.ids gpurun_out/${T}_c5_g$g.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
done
