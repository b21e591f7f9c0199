#!/bin/bash
# Round 5: the 16-slot active-set kernels.  Their parity tests first, then the whole GPU suite,
# the three-contact bench line on the active-set path and on the interior point kernel alone
# (kernel traces of both), and the default bench line.  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05d}
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_contact.py tests/test_gpu_c5_windows.py tests/test_gpu_dcm_mpc.py tests/test_gpu_phased.py -v -x -m gpu --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest_mc.log 2>&1
rc=$?; grep -E "FAILED|ERROR|Error" gpurun_out/${T}_pytest_mc.log | head -5; tail -1 gpurun_out/${T}_pytest_mc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload mc --steps 10 --warmup 3 > gpurun_out/${T}_bench_mc.log 2>&1 || { echo "mc failed"; tail -5 gpurun_out/${T}_bench_mc.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench_mc.log | tail -1 | cut -c1-400
BLF_QP_SINGLE_KERNEL=1 timeout -k 10 300 python bench.py --workload mc --steps 10 --warmup 3 --expand-path > gpurun_out/${T}_bench_mc_ipm.log 2>&1 || { echo "mc ipm failed"; tail -5 gpurun_out/${T}_bench_mc_ipm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench_mc_ipm.log | tail -1 | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_mc_trace -o run -- python3 bench.py --workload mc --steps 5 --warmup 2 > gpurun_out/${T}_mc_trace.log 2>&1 || { echo "mc trace failed"; exit 1; }
BLF_QP_SINGLE_KERNEL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${T}_mc_ipm_trace -o run -- python3 bench.py --workload mc --steps 5 --warmup 2 --expand-path > gpurun_out/${T}_mc_ipm_trace.log 2>&1 || { echo "mc ipm trace failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench.log | tail -1 | cut -c1-300
