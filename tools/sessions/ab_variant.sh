#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/kbench.py --reps 20 > gpurun_out/kb_base.log 2>&1 || exit 1
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_variant.so timeout -k 10 200 python tools/kbench.py --reps 20 > gpurun_out/kb_fma.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/kb_base.log | tail -3; grep -v amdgpu gpurun_out/kb_fma.log | tail -3
