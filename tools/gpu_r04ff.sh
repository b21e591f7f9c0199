#!/bin/bash
# Round 4: the c5 overlap path (deferred stage 2 on a side stream) on the final build, against the
# default two groups, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "2 0" "1 1" "2 1"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $1 --c5-overlap $2 > gpurun_out/r04ff_c5_g$1_o$2_$r.log 2>&1 || { echo "c5 g=$1 o=$2 failed"; exit 1; }
    echo -n "c5 groups=$1 overlap=$2 round $r: "; grep -v amdgpu.ids gpurun_out/r04ff_c5_g$1_o$2_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done | tee gpurun_out/r04ff_c5_overlap.log
