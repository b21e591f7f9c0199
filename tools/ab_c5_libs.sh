#!/bin/bash
# A/B of library builds on the closed loop (bench.py --workload c5, CPU baseline off), ROUNDS
# alternations:  LIBS="libblf.so libblf_x.so" ROUNDS=2 TAG=r06x tools/ab_c5_libs.sh
# -> gpurun_out/$TAG_c5_ab.log (ms_per_step and the QP status counts per run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LOG=gpurun_out/${TAG:-ab}_c5_ab.log
: > $LOG
for r in $(seq ${ROUNDS:-2}); do
  for l in ${LIBS:-libblf.so}; do
    BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$l timeout -k 10 200 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu \
        > gpurun_out/c5_ab_run.log 2>&1 || { echo "c5 $l failed"; tail -5 gpurun_out/c5_ab_run.log; exit 1; }
    echo "round $r $l $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_ab_run.log) $(grep -o '"qp_status_counts": {[^}]*}' gpurun_out/c5_ab_run.log)" >> $LOG
  done
done
cat $LOG
