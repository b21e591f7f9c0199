#!/bin/bash
# Round 4 diagnostics: the hard c5 windows on the stamp build (IPM kernel phases of one window).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
BLF_LIB=$L/libblf_stamps.so timeout -k 10 120 python tools/hard_windows_timing.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04h_hard_stamps.log || exit 1
