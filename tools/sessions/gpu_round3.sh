#!/bin/bash
# Round-3 evidence on one GPU box: the default bench line, the other workloads (c1 c3 c5 rh) and
# the batch-scaling kbench, the rocprofv3 passes of the headline (tools/profile_round.sh), the
# fbd per-phase stamps.  Each GPU step under its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-300
bash tools/sessions/gpu_workloads.sh || exit 1
if [ "${PROFILE:-1}" = 1 ]; then
  bash tools/profile_round.sh > gpurun_out/profile.log 2>&1 || { echo "profile failed"; exit 1; }
fi
if [ -f bipedal-locomotion-framework_amd/lib/libblf_stamps.so ] && [ "${STAMPS:-1}" = 1 ]; then
  BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_stamps.so timeout -k 10 120 python tools/fbd_stamps.py > gpurun_out/fbd_stamps.log 2>&1 || { echo "stamps failed"; exit 1; }
fi
echo done
