#!/bin/bash
# Diagnostics: event-timed median of one streaming kernel (STREAM_KERNEL, default rollout) with the
# product library and every lib/libblf_<name>.so variant, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in bipedal-locomotion-framework_amd/lib/libblf.so bipedal-locomotion-framework_amd/lib/libblf_[pv]*.so; do
    STREAM_TIME=1 BLF_LIB=$PWD/$lib timeout -k 10 120 python tools/stream_one.py ${STREAM_KERNEL:-rollout} 2>&1 | grep -v amdgpu.ids || exit 1
done
