#!/bin/bash
# Round 4: the dynamics kernel's own-pivot capture and fma substitutions (BLF_FBD_DIAGCAP):
# fb / closed-loop GPU tests on the variant, then two rounds of one c5 period against the shipped
# build (libblf_dc0 = the build profiled in profiles/r04_v6_*).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T=${TAG:-r04aa}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fb_dynamics.py tests/test_gpu_closed_loop.py \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
L=$PWD/bipedal-locomotion-framework_amd/lib
for r in 1 2 3; do
  for lib in libblf libblf_dc0; do
    echo -n "$lib: "
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/${T}_ab.log
