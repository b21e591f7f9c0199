#!/bin/bash
# Round 4 evidence on the shipped build: the bench's kernel trace and PMC passes
# (tools/profile_round.sh), the streaming kernels' trace and HBM passes (tools/gpu_stream.sh), and
# the SQ passes of fbd_euler_kernel (tools/gpu_sq.sh).  Every summary records the library hash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 1500 bash tools/profile_round.sh > gpurun_out/prof_round.log 2>&1 || { echo "profile_round failed"; tail -5 gpurun_out/prof_round.log; exit 1; }
echo "profile_round done"
timeout -k 10 900 bash tools/gpu_stream.sh > gpurun_out/prof_stream.log 2>&1 || { echo "stream failed"; tail -5 gpurun_out/prof_stream.log; exit 1; }
echo "stream done"
KERNELS=fbd_euler SQ_EXTRA=1 timeout -k 10 1200 bash tools/gpu_sq.sh > gpurun_out/prof_sq.log 2>&1 || { echo "sq failed"; tail -5 gpurun_out/prof_sq.log; exit 1; }
echo "sq done"
