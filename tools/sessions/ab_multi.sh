#!/bin/bash
# Diagnostics: kbench on the product library and every lib/libblf_<name>.so variant
# (tools/build_variant.sh), each under its own time limit.  KB_ARGS passes kbench options.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
out=gpurun_out/ab_multi.log
: > $out
for lib in bipedal-locomotion-framework_amd/lib/libblf.so bipedal-locomotion-framework_amd/lib/libblf_v*.so; do
    BLF_LIB=$PWD/$lib timeout -k 10 120 python tools/kbench.py ${KB_ARGS:---reps 20 --tol-polish 0 1e-6} 2>&1 | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
