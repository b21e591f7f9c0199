#!/bin/bash
# Round 4: the overlap test, the c5 line without / with the overlap (CU-partitioned streams), two
# rounds, and a kernel trace of the overlap.  Each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04n}
timeout -k 10 300 python -u -m pytest tests/test_gpu_closed_loop.py -v -m gpu -k "overlap or groups" --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${T}_pytest.log | tail -4
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for o in 0 1; do
    timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-overlap $o > gpurun_out/${T}_c5_o${o}_$r.log 2>&1 || { echo "c5 o=$o failed"; exit 1; }
    echo -n "overlap=$o round $r: "; grep -v amdgpu.ids gpurun_out/${T}_c5_o${o}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_trace -o run -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu --c5-overlap 1 > gpurun_out/${T}_trace.log 2>&1 || exit 1
f=$(find gpurun_out/${T}_trace -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/${T}_kernel_trace.csv
