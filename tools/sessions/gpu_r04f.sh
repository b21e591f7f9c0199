#!/bin/bash
# Round 4: the c5 line at 1 / 2 / 3 stream groups, two rounds; each run under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for r in 1 2; do
  for g in ${GROUPS_LIST:-1 2 3}; do
    timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/r04f_c5_g${g}_$r.log 2>&1 || { echo "c5 g=$g failed"; exit 1; }
    echo -n "groups=$g round $r: "; grep -v amdgpu.ids gpurun_out/r04f_c5_g${g}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done
