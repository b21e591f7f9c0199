#!/bin/bash
# Round 4: the c5 line at two, three and four stream groups on the final build, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for r in 1 2; do
  for g in 2 3 4; do
    timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/r04dd_c5_g${g}_$r.log 2>&1 || { echo "c5 g=$g failed"; exit 1; }
    echo -n "c5 groups=$g round $r: "; grep -v amdgpu.ids gpurun_out/r04dd_c5_g${g}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done | tee gpurun_out/r04dd_c5_groups.log
