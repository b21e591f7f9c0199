#!/bin/bash
# Round 4: QP parity tests (c5 windows, phased, dcm_mpc, multi-contact), the hard-window timing,
# the cold QP kernel's stamps at 4096 QPs, kbench.  Each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
T=${TAG:-r04q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_windows.py tests/test_gpu_phased.py tests/test_gpu_dcm_mpc.py tests/test_gpu_multi_contact.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${T}_pytest.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/hard_windows_timing.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_hard.log || exit 1
[ -f $L/libblf_stamps.so ] && { BLF_LIB=$L/libblf_stamps.so timeout -k 10 120 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids > gpurun_out/${T}_kb_stamps.log || exit 1; tail -12 gpurun_out/${T}_kb_stamps.log; }
timeout -k 10 120 python tools/kbench.py --reps 20 2>&1 | grep -v amdgpu.ids | tail -1
