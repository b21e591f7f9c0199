#!/bin/bash
# A/B of library builds on one box (tools/kbench.py, HIP events, configs[1] by default):
#   LIBS="libblf.so libblf_x.so libblf.so:BLF_QP_FUSE_STAGE2=0 ..." ROUNDS=2 TAG=r06x tools/gpu_ab_libs.sh [kbench args...]
# Every library in turn (an entry lib:VAR=value runs it with that environment variable set),
# ROUNDS times, into gpurun_out/$TAG_ab.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LOG=gpurun_out/${TAG:-ab}_ab.log
: > $LOG
for r in $(seq ${ROUNDS:-2}); do
  for l in ${LIBS:-libblf.so}; do
    echo "== round $r $l" >> $LOG
    lib=${l%%:*}; ev=""; [ "$lib" != "$l" ] && ev=${l#*:}
    env $ev BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/$lib timeout -k 10 200 python tools/kbench.py "$@" 2>&1 | grep -v amdgpu.ids >> $LOG \
      || { echo "kbench $l failed"; tail -5 $LOG; exit 1; }
  done
done
cat $LOG
