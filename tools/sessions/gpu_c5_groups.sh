#!/bin/bash
# c5 stream groups: the bitwise test, then the bench at 1 / 2 / 4 groups (two rounds, one box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_closed_loop.py > gpurun_out/cl_tests.log 2>&1 || { tail -20 gpurun_out/cl_tests.log; exit 1; }
tail -1 gpurun_out/cl_tests.log
for r in 1 2; do
  for g in 1 2 4; do
    timeout -k 10 200 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/c5_g$g.log 2>&1 || exit 1
    echo "c5 groups $g: $(grep -v amdgpu.ids gpurun_out/c5_g$g.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"], 3), "ms", round(d["value"]), d["qp_status_counts"])')"
  done
done
