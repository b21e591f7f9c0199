#!/bin/bash
# Round 5: config-5 closed loop on the current build: bench lines at one and two stream groups and
# a kernel trace of the default (two groups).  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05e}
for g in 2 1; do
  timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/${T}_c5_g$g.log 2>&1 || { echo "c5 g=$g failed"; tail -3 gpurun_out/${T}_c5_g$g.log; exit 1; }
  echo -n "c5 groups=$g: "; grep -v amdgpu.ids gpurun_out/${T}_c5_g$g.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_c5_trace -o run -- python3 bench.py --workload c5 --no-cpu --steps 6 --warmup 2 > gpurun_out/${T}_c5_trace.log 2>&1 || { echo "trace failed"; exit 1; }
cat $(find gpurun_out/${T}_c5_trace -name "*kernel_stats.csv") | cut -d, -f1-4,6,7 | head -12
