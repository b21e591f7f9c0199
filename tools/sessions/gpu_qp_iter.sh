#!/bin/bash
# QP kernel iteration on one GPU box: the QP parity tests, kbench timings at 1536 / 4096 / 65536,
# and the stamp build's per-phase cycles at 4096.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dcm_mpc.py tests/test_gpu_receding_horizon.py tests/test_gpu_closed_loop.py > gpurun_out/qp_tests.log 2>&1
rc=$?; echo "qp tests rc=$rc"; tail -3 gpurun_out/qp_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 1536 4096 65536; do
    timeout -k 10 100 python tools/kbench.py --reps 20 --batch $b 2>&1 | grep -v amdgpu.ids || exit 1
done
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_stamps.so timeout -k 10 100 python tools/kbench.py --reps 10 --batch 4096 2>&1 | grep -v amdgpu.ids || exit 1
