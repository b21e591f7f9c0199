#!/bin/bash
# Round 4: the floating-base / closed-loop / host GPU tests on the current build, then an
# event-timed A/B of fbd_euler_kernel (product vs lib/libblf_<name>.so in $LIBS, alternating,
# $ROUNDS rounds), then the c5 bench line.  Each GPU step under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T=${TAG:-r04b}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_fb_dynamics.py tests/test_host_cpp.py tests/test_gpu_closed_loop.py} -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest.log | head -10; tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in $(seq ${ROUNDS:-2}); do
  for lib in libblf ${LIBS:-}; do
    for k in ${TIME_KERNELS:-fbd_euler}; do
      echo -n "$lib $k: "
      BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$lib.so STREAM_TIME=1 timeout -k 10 120 python tools/stream_one.py $k 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done | tee gpurun_out/${T}_ab.log
[ "${C5:-1}" = 1 ] || exit 0
timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/${T}_bench_c5.log 2>&1 || { echo "c5 failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bench_c5.log | tail -1 | cut -c1-400
