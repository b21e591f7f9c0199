#!/bin/bash
# HBM roofline of the streaming kernels: event timing, then rocprofv3 kernel trace and the
# FETCH_SIZE / WRITE_SIZE passes of the same run (separate passes, MI355X_MICROARCH.md HBM section).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/stream_prof
mkdir -p $OUT
timeout -k 10 120 python3 -c "import json, sys; sys.path.insert(0, 'bipedal-locomotion-framework_amd'); from blf import native; print(json.dumps(native.build_provenance()))" > $OUT/build.json || exit $?
export TMPDIR=/tmp
timeout -k 10 300 python tools/stream_bench.py --out gpurun_out/stream.json > gpurun_out/stream.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stream.log | tail -8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 tools/stream_bench.py > $OUT/trace.log 2>&1 || exit $?
if [ "${STREAM_PMC:-1}" = 1 ]; then
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run -- python3 tools/stream_bench.py > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run -- python3 tools/stream_bench.py > $OUT/write.log 2>&1 || exit $?
fi
f=$(find $OUT/trace -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f"
exit 0
