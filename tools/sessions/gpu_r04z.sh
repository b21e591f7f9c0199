#!/bin/bash
# Round 4: the dynamics kernel's per-system constant staging (BLF_FBD_CSTAGE) and the QP kernels'
# per-pass opaque lane index (BLF_AS_OPQLANE): fb / closed-loop / QP GPU tests on the product, then
# two rounds of each A/B on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T=${TAG:-r04z}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fb_dynamics.py tests/test_gpu_closed_loop.py tests/test_gpu_contact.py \
  tests/test_gpu_dcm_mpc.py tests/test_gpu_receding_horizon.py tests/test_gpu_qp_split.py \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
L=$PWD/bipedal-locomotion-framework_amd/lib
for r in 1 2; do
  for lib in libblf libblf_cs0; do
    echo -n "$lib: "
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
  for lib in libblf libblf_vopq0; do
    for b in 4096 65536; do
      BLF_LIB=$L/$lib.so timeout -k 10 100 python tools/kbench.py --reps 20 --batch $b 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done | tee gpurun_out/${T}_ab.log
