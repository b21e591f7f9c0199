#!/bin/bash
# Round 4: the pointer-jumping kinematics (BLF_FBD_KINJUMP) -- fb / closed-loop GPU tests on the
# product build, then one c5 period of fbd_euler_kernel against the level-recursion build and the
# LDS model-copy build, two rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T=${TAG:-r04t}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fb_dynamics.py tests/test_gpu_closed_loop.py tests/test_gpu_contact.py \
  > gpurun_out/${T}_pytest_fb.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_fb.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_fb.log
L=$PWD/bipedal-locomotion-framework_amd/lib
for r in 1 2; do
  for lib in libblf ${LIBS:-libblf_kinlev libblf_ldsm}; do
    echo -n "$lib: "
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/${T}_fbd_ab.log
BLF_LIB=$L/libblf_stamps.so timeout -k 10 120 python tools/fbd_stamps.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${T}_fbd_stamps.log
