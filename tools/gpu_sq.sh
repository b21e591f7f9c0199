#!/bin/bash
# SQ counter passes (one rocprofv3 run per counter group) for the streaming kernels named in $KERNELS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sq
mkdir -p $OUT
export TMPDIR=/tmp
for k in ${KERNELS:-rollout hull}; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $grp -T --output-format csv -d $OUT/$k$i -o run -- python3 tools/stream_one.py $k > $OUT/$k$i.log 2>&1 || { echo "fail $k $grp"; tail -5 $OUT/$k$i.log; exit 1; }
  done
done
echo done
