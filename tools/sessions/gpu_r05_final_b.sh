#!/bin/bash
# Round 5 final build: rocprofv3 evidence -- the c2 kernel trace and PMC passes (profile_round.sh),
# the streaming kernels (gpu_stream.sh), the fbd_euler SQ passes, the c5 / c3 / rh kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash tools/profile_round.sh > gpurun_out/r05fb_prof_round.log 2>&1 || { echo "profile_round failed"; tail -5 gpurun_out/r05fb_prof_round.log; exit 1; }
echo profile_round done
bash tools/gpu_stream.sh > gpurun_out/r05fb_stream.log 2>&1 || { echo "stream failed"; tail -5 gpurun_out/r05fb_stream.log; exit 1; }
echo stream done
KERNELS=fbd_euler SQ_EXTRA=1 bash tools/gpu_sq.sh > gpurun_out/r05fb_sq.log 2>&1 || { echo "sq failed"; tail -5 gpurun_out/r05fb_sq.log; exit 1; }
echo sq done
WORKLOADS="c5 c3 rh" bash tools/gpu_ktrace_workloads.sh > gpurun_out/r05fb_ktw.log 2>&1 || { echo "ktw failed"; tail -5 gpurun_out/r05fb_ktw.log; exit 1; }
cat gpurun_out/r05fb_ktw.log
