#!/bin/bash
# Round 4: the c5 line with the overlap in three CU layouts (side stream on 8 CUs of its own, the
# main stream everywhere / split / no masks) against no overlap, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r04o}
for r in 1 2; do
  for cfg in 0:none 1:side 1:none 1:split; do
    o=${cfg%%:*}; m=${cfg##*:}
    BLF_OVERLAP_CU_MODE=$m timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-overlap $o > gpurun_out/${T}_c5_${o}_${m}_$r.log 2>&1 || { echo "c5 $cfg failed"; exit 1; }
    echo -n "overlap=$o cu=$m round $r: "; grep -v amdgpu.ids gpurun_out/${T}_c5_${o}_${m}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done
