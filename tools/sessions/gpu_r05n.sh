#!/bin/bash
# c5 period vs the number of stream groups (the closed loops' overlap), with the ABA layout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 1 2 3 4 2; do
  timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/r05n_c5_g$g.log 2>&1 || { echo "c5 g=$g failed"; tail -3 gpurun_out/r05n_c5_g$g.log; exit 1; }
  echo -n "groups=$g: "; grep -v amdgpu.ids gpurun_out/r05n_c5_g$g.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
done
