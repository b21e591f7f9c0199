#!/bin/bash
# A/B of BLF_AS_KEEPIN (phase B reuses phase A's fp64 knot inputs) on the configs[1] bench:
# product vs lib/libblf_vkin0.so, alternating, three rounds; then the QP bitwise tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/bipedal-locomotion-framework_amd/lib/libblf_vkin0.so
for r in 1 2 3; do
  for lib in keep reload; do
    if [ $lib = keep ]; then unset BLF_LIB; else export BLF_LIB=$V; fi
    timeout -k 10 300 python bench.py --no-cpu --steps 50 > gpurun_out/r05s_${lib}_$r.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/r05s_${lib}_$r.log; exit 1; }
    echo -n "$lib $r: "; grep -v amdgpu.ids gpurun_out/r05s_${lib}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
unset BLF_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_dcm_mpc.py tests/test_gpu_kernels.py -q -x -m gpu --timeout 300 --timeout-method thread 2>&1 | tail -2
