#!/bin/bash
# Round 4: the overlap test, the c5 line without / with the overlap (high-priority side stream),
# two rounds, and the fbd_euler A/B against $FBD_LIBS.  Each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
T=${TAG:-r04j}
timeout -k 10 300 python -u -m pytest tests/test_gpu_closed_loop.py -v -m gpu -k overlap --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${T}_pytest.log | tail -4
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for o in ${OVERLAPS:-0 1}; do
    timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-overlap $o ${C5_ARGS:-} > gpurun_out/${T}_c5_o${o}_$r.log 2>&1 || { echo "c5 o=$o failed"; exit 1; }
    echo -n "overlap=$o round $r: "; grep -v amdgpu.ids gpurun_out/${T}_c5_o${o}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done
for r in 1 2; do
  for lib in libblf ${FBD_LIBS:-}; do
    echo -n "$lib fbd_euler: "
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/${T}_fbd_ab.log
