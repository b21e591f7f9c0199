#!/bin/bash
# Round 4 diagnostics: warm solves of the committed hard c5 windows, event-timed, then under a
# kernel trace.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/hard_windows_timing.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04g_hard.log || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/r04g_prof -o run -- python3 tools/hard_windows_timing.py > gpurun_out/r04g_prof.log 2>&1 || exit 1
f=$(find gpurun_out/r04g_prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -8
