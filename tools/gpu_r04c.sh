#!/bin/bash
# Round 4: the whole GPU suite on the current build (split QP kernels, folded fbd substitution),
# then event-timed A/Bs: fbd_euler_kernel (product vs $FBD_LIBS) and the cold QP kernels fused vs
# split (BLF_QP_SPLIT_MIN_BATCH) at 4096 / 65 536 QPs, then the c5 line.  Each GPU step under its
# own time limit; a crash or time limit ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${TAG:-r04c}
L=$PWD/bipedal-locomotion-framework_amd/lib
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -v --maxfail=5 -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -10; tail -2 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
[ "${SKIP_FBD:-0}" = 1 ] || for r in 1 2; do
  for lib in libblf ${FBD_LIBS:-}; do
    echo -n "$lib fbd_euler: "
    BLF_LIB=$L/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py fbd_euler 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee gpurun_out/${T}_fbd_ab.log
for r in 1 2; do
  for B in ${QP_BATCHES:-4096 65536}; do
    for cfg in libblf:0 libblf:1 ${QP_EXTRA:-}; do   # lib:split_min_batch
      lib=${cfg%%:*}; sm=${cfg##*:}
      echo -n "$lib split_min=$sm B=$B: "
      BLF_LIB=$L/$lib.so BLF_QP_SPLIT_MIN_BATCH=$sm timeout -k 10 120 python tools/kbench.py --batch $B --reps 20 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done | tee gpurun_out/${T}_split_ab.log
[ "${SKIP_C5:-0}" = 1 ] && exit 0
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/${T}_bench_c5.log 2>&1 || { echo "c5 failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench_c5.log | tail -1 | cut -c1-400
