#!/bin/bash
# Round 4 diagnostics: the cold QP kernel's phase stamps and wave timeline at 4096 QPs (stamp build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
BLF_LIB=$L/libblf_stamps.so timeout -k 10 120 python tools/kbench.py --reps 3 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04p_kb_stamps.log || exit 1
timeout -k 10 120 python tools/kbench.py --reps 20 2>&1 | grep -v amdgpu.ids | tail -2
