#!/bin/bash
# A/B of the Riccati element forms (BLF_RC_FORM, csrc/dcm_qp_common.h): kbench on the product
# library and the lib/libblf_vrc<form>.so variants, ROUNDS rounds alternating the libraries, at
# configs[0] (B = 1, N = 50), the headline (B = 4096, N = 100) and a large batch (65 536).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
out=gpurun_out/rc_ab.log
: > $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in libblf ${LIBS:-libblf_vrc1 libblf_vrc2 libblf_vrc3}; do
    for cfg in "--batch 1 --horizon 50 --reps 200" "--batch 4096 --horizon 100 --reps 50" "--batch 65536 --horizon 100 --reps 10"; do
      BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$lib.so timeout -k 10 120 python tools/kbench.py $cfg 2>&1 | grep -v amdgpu.ids >> $out || exit 1
    done
  done
done
cat $out
