#!/bin/bash
# Diagnostics: kbench of the product library and every lib/libblf_<name>.so named in $LIBS at the
# batch sizes in $BATCHES (each GPU step under its own time limit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for lib in libblf ${LIBS:-}; do
    for b in ${BATCHES:-4096}; do
        BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$lib.so timeout -k 10 100 python tools/kbench.py --reps 20 --batch $b 2>&1 | grep -v amdgpu.ids || exit 1
    done
done
