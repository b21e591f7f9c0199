#!/bin/bash
# Six lanes per joint in the articulated-body sweeps (fbd_aba_rows): fb / closed-loop / host tests,
# then fbd_euler product vs lib/libblf_vlane.so (one lane per joint) and the c5 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fb_dynamics.py tests/test_gpu_closed_loop.py tests/test_host_cpp.py tests/test_gpu_urdf.py -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR|assert" gpurun_out/${T}_pytest_gpu.log | head -20; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids || exit 1
  BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_vlane.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids || exit 1
done
for r in 1 2; do
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/${T}_c5_$r.log 2>&1 || { echo "c5 failed"; tail -3 gpurun_out/${T}_c5_$r.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_c5_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
done
