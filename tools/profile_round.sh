#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats of the bench command, then separate
# PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Run on the GPU box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 120 python3 -c "import json, sys; sys.path.insert(0, 'bipedal-locomotion-framework_amd'); from blf import native; print(json.dumps(native.build_provenance()))" > $OUT/build.json || exit $?
BENCH="bench.py --steps 10 --warmup 2 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run -- python3 $BENCH > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run -- python3 $BENCH > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T --output-format csv -d $OUT/sq -o run -- python3 $BENCH > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -T --output-format csv -d $OUT/sq2 -o run -- python3 $BENCH > $OUT/sq2.log 2>&1 || exit $?
# the stall breakdown (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES) and LDS detail
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA -T --output-format csv -d $OUT/sq3 -o run -- python3 $BENCH > $OUT/sq3.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -50
