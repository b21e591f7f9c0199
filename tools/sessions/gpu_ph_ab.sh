#!/bin/bash
# Phase-indexed cold staging overlap: QP parity tests, then c3 / rh A/B against lib/libblf_ph0.so.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_phased.py tests/test_gpu_pipeline_c3.py tests/test_gpu_dcm_mpc.py tests/test_gpu_receding_horizon.py > gpurun_out/ph_tests.log 2>&1 || { tail -20 gpurun_out/ph_tests.log; exit 1; }
tail -1 gpurun_out/ph_tests.log
for r in 1 2; do
  for v in libblf.so libblf_ph0.so; do
    BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$v timeout -k 10 200 python bench.py --workload c3 --no-cpu > gpurun_out/c3_$v.log 2>&1 || exit 1
    echo "c3 $v: $(grep -v amdgpu.ids gpurun_out/c3_$v.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"], 4), "ms", round(d["value"]))')"
  done
done
