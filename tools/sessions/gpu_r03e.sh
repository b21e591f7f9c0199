#!/bin/bash
# fbd blocked substitutions (parity tests, then Euler-kernel A/B against one unknown per step) and
# the phase-expansion non-temporal store A/B on the two-call receding-horizon path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fb_dynamics.py tests/test_gpu_closed_loop.py > gpurun_out/fbd_tests.log 2>&1 || { tail -20 gpurun_out/fbd_tests.log; exit 1; }
tail -1 gpurun_out/fbd_tests.log
for r in 1 2; do
  for v in sub2 sub1 cb4; do
    STREAM_TIME=1 BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_$v.so timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
for r in 1 2; do
  for v in pent1 pent0; do
    BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_$v.so timeout -k 10 200 python bench.py --workload rh --expand-path --no-cpu > gpurun_out/rh_$v.log 2>&1 || exit 1
    echo "rh --expand-path $v: $(grep -v amdgpu.ids gpurun_out/rh_$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
for v in pent1 pent0; do
  BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_$v.so timeout -k 10 200 python bench.py --workload c3 --expand-path --no-cpu > gpurun_out/c3_$v.log 2>&1 || exit 1
  echo "c3 --expand-path $v: $(grep -v amdgpu.ids gpurun_out/c3_$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
for r in 1 2; do
  for v in hull1 hull0; do
    STREAM_TIME=1 BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_$v.so timeout -k 10 120 python tools/stream_one.py hull 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
echo done
