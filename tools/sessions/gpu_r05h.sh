#!/bin/bash
# Round 5: contact laws (blf_fb_contacts.law, blf_fb_frame_state): the floating-base GPU tests and
# the C++ host tests, then the c5 bench line (the fbd kernels gained the law branch).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fb_dynamics.py tests/test_host_cpp.py tests/test_gpu_closed_loop.py -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR|Error|assert" gpurun_out/${T}_pytest_gpu.log | head -20; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/${T}_c5.log 2>&1 || { echo "c5 failed"; tail -3 gpurun_out/${T}_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_c5.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
