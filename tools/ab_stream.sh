#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/stream_bench.py > gpurun_out/sb_base.log 2>&1 || exit 1
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_variant.so timeout -k 10 200 python tools/stream_bench.py > gpurun_out/sb_var.log 2>&1 || exit 1
grep rollout gpurun_out/sb_base.log | cut -c1-120; grep rollout gpurun_out/sb_var.log | cut -c1-120
