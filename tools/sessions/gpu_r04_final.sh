#!/bin/bash
# Round 4, final build: the whole GPU suite, the bench lines of every workload, and the c5 line at
# one and two stream groups (two rounds).  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T=${TAG:-r04f1}
timeout -k 10 900 python -u -m pytest tests -v --maxfail=5 -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -2 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in c2 c1 c3 rh; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/${T}_bench_$w.log 2>&1 || { echo "bench $w failed"; exit 1; }
  echo -n "$w: "; grep -v amdgpu.ids gpurun_out/${T}_bench_$w.log | tail -1 | cut -c1-160
done
for r in 1 2; do
  for g in 1 2; do
    timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/${T}_c5_g${g}_$r.log 2>&1 || { echo "c5 g=$g failed"; exit 1; }
    echo -n "c5 groups=$g round $r: "; grep -v amdgpu.ids gpurun_out/${T}_c5_g${g}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done
timeout -k 10 300 python tools/kbench.py --batch 65536 --reps 10 2>&1 | grep -v amdgpu.ids | tail -1
