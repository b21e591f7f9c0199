#!/bin/bash
# Round-3 evidence run 2 of 2: the headline's rocprofv3 passes (tools/profile_round.sh), the
# streaming kernels' HBM passes (tools/gpu_stream.sh), SQ passes of hull2d and the fbd Euler kernel,
# the fbd per-phase stamps.  Each step under its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
bash tools/profile_round.sh > gpurun_out/profile.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/profile.log; exit 1; }
echo profile ok
bash tools/gpu_stream.sh > gpurun_out/stream_run.log 2>&1 || { echo "stream failed"; tail -5 gpurun_out/stream_run.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stream.log | tail -8
KERNELS="hull fbd_euler" SQ_EXTRA=1 bash tools/gpu_sq.sh > gpurun_out/sq_run.log 2>&1 || { echo "sq failed"; tail -5 gpurun_out/sq_run.log; exit 1; }
echo sq ok
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_stamps.so timeout -k 10 120 python tools/fbd_stamps.py > gpurun_out/fbd_stamps.log 2>&1 || { echo "fbd stamps failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/fbd_stamps.log | tail -12
echo done
