#!/bin/bash
# Round 5: stage-2 list grid A/B (kernel trace of the default bench per grid), then the whole GPU
# suite and the default bench line.  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05c}
for G in 1 16 64 256 1024; do
  BLF_QP_LIST_GRID=$G timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_g$G -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/${T}_g$G.log 2>&1 || { echo "grid $G failed"; exit 1; }
  echo -n "grid $G: "; grep -h "dcm_mpc_ipm_list_kernel\|dcm_mpc_cold_kernel" $(find gpurun_out/${T}_g$G -name "*kernel_stats.csv") | cut -d, -f1,2,4,6 | tr '\n' ' '; echo
done
timeout -k 10 900 python -u -m pytest tests -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench.log | tail -1 | cut -c1-300
