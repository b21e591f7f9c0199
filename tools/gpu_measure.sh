#!/bin/bash
# One measurement session on the GPU box, every step under its own time limit, the first failure
# ends it:  TAG=r06x tools/gpu_measure.sh [tests] [bench] [sqfbd] [ktrace_c5]
#   tests      pytest -m gpu                         -> gpurun_out/$TAG_pytest_gpu.log
#   bench      bench.py lines c2 (default), c5, mc, rh, c1, c3 (CPU baselines included)
#                                                    -> gpurun_out/$TAG_bench_<w>.log
#   sqfbd      SQ counter passes of fbd_euler_kernel (tools/gpu_sq.sh, SQ_EXTRA=1) and their
#              summary                              -> gpurun_out/$TAG_fbd_euler_sq.json
#   ktrace_c5  rocprofv3 kernel trace + stats of the c5 bench -> gpurun_out/$TAG_ktrace_c5/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
          -p no:cacheprovider > gpurun_out/${TAG}_pytest_gpu.log 2>&1
      rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc = 0 ] || { echo "tests rc=$rc"; exit $rc; } ;;
    bench)
      for w in ${WORKLOADS:-c2 c5 mc rh c1 c3}; do
        timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/${TAG}_bench_$w.log 2>&1 \
            || { echo "bench $w failed"; tail -5 gpurun_out/${TAG}_bench_$w.log; exit 1; }
        echo "$w: $(grep -v amdgpu.ids gpurun_out/${TAG}_bench_$w.log | tail -1 | cut -c1-300)"
      done ;;
    sqfbd)
      rm -rf gpurun_out/sq
      SQ_EXTRA=1 KERNELS=fbd_euler bash tools/gpu_sq.sh || exit 1
      python tools/sq_summary.py fbd_euler fbd_euler_kernel gpurun_out/${TAG}_fbd_euler_sq.json > /dev/null || exit 1
      echo "sqfbd: gpurun_out/${TAG}_fbd_euler_sq.json" ;;
    ktrace_c5)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/${TAG}_ktrace_c5 -o run \
          -- python3 bench.py --workload c5 --steps 6 --warmup 2 --no-cpu > gpurun_out/${TAG}_ktrace_c5.log 2>&1 \
          || { echo "ktrace_c5 failed"; exit 1; }
      echo "ktrace_c5: $(ls gpurun_out/${TAG}_ktrace_c5 | head -3)" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu_measure done"
