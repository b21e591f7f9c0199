#!/bin/bash
# Round 4: the fp32 search's hand-over threshold (kHandoverDiv: N / 8, N / 12, N / 24 against the
# shipped N / 16), kbench at 4096 and 65 536 QPs, two rounds on one box (timing only: the variants
# are not matched by the oracle).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
for r in 1 2; do
  for lib in libblf libblf_vho8 libblf_vho12 libblf_vho24; do
    for b in 4096 65536; do
      echo -n "$lib: "
      BLF_LIB=$L/$lib.so timeout -k 10 100 python tools/kbench.py --reps 20 --batch $b 2>&1 | grep -v amdgpu.ids | tail -1 | sed 's/.*batch=/batch=/' || exit 1
    done
  done
done | tee gpurun_out/r04cc_handover_ab.log
