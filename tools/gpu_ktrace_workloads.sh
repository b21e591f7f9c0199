#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of the bench's secondary workloads (c3
# pipeline, c5 closed loop, rh receding horizon), CPU baselines off.  Results in gpurun_out/ktw_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in ${WORKLOADS:-c3 c5 rh}; do
    tag=ktw_$w
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -T --output-format csv \
        -d gpurun_out/$tag -o run -- python3 bench.py --workload $w --steps 5 --warmup 1 --no-cpu \
        > gpurun_out/$tag.log 2>&1 || exit $?
    echo "== $tag"
    f=$(find gpurun_out/$tag -name "*kernel_stats.csv" | head -1)
    cp "$f" gpurun_out/${tag}_kernel_stats.csv
    cut -d, -f1-5 "$f" | head -8
done
