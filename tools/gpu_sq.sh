#!/bin/bash
# SQ counter passes (one rocprofv3 run per counter group) for the targets named in $KERNELS:
# streaming kernels (tools/stream_one.py) or the QP kernel ("ipm": tools/kbench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 -c "import json, sys; sys.path.insert(0, 'bipedal-locomotion-framework_amd'); from blf import native; print(json.dumps(native.build_provenance()))" > $OUT/build.json || exit $?
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
)
if [ "${SQ_EXTRA:-0}" = 1 ]; then
  GROUPS_+=(
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
    "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
    "SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_SMEM"
  )
fi
for k in ${KERNELS:-rollout hull}; do
  if [ "$k" = ipm ]; then CMD="tools/kbench.py --reps 3"; else CMD="tools/stream_one.py $k"; fi
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $grp -T --output-format csv -d $OUT/$k$i -o run -- python3 $CMD > $OUT/$k$i.log 2>&1 || { echo "fail $k $grp"; tail -5 $OUT/$k$i.log; exit 1; }
  done
done
echo done
