#!/bin/bash
# A/B of the closed loop's cold-after-hand-over rule on the c5 bench, alternating, three rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 1 0; do
    BLF_C5_COLD_AFTER_HANDOVER=$v timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/r05r_c5_${v}_$r.log 2>&1 || { echo "c5 failed"; exit 1; }
    echo -n "cold_after_handover=$v round $r: "; grep -v amdgpu.ids gpurun_out/r05r_c5_${v}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done
