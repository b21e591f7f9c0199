#!/bin/bash
# Per-kernel times (rocprofv3 --kernel-trace --stats) of tools/kbench.py at a few batch sizes, with
# the default two-kernel QP path and with BLF_QP_SINGLE_KERNEL=1.  Results in gpurun_out/kt_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${BATCHES:-4096 65536}; do
  for single in 0 1; do
    tag=kt_${b}_s${single}
    BLF_QP_SINGLE_KERNEL=$single timeout -k 10 120 rocprofv3 --kernel-trace --stats -T --output-format csv \
        -d gpurun_out/$tag -o run -- python3 tools/kbench.py --batch $b --reps 10 > gpurun_out/$tag.log 2>&1 || exit $?
    echo "== $tag"; grep -v amdgpu.ids gpurun_out/$tag.log | tail -1
    f=$(find gpurun_out/$tag -name "*kernel_stats.csv" | head -1)
    cut -d, -f1-4 "$f" | head -6
  done
done
