#!/bin/bash
# Instruction-cache counters of the QP kernel (kbench, B=4096), one rocprofv3 --pmc pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/icpmc
mkdir -p $OUT
KB="tools/kbench.py --reps 5 --batch ${KB_BATCH:-4096}"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY -T --output-format csv -d $OUT/p1 -o run -- python3 $KB > $OUT/p1.log 2>&1 || { echo "pass failed"; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VALU -T --output-format csv -d $OUT/p2 -o run -- python3 $KB > $OUT/p2.log 2>&1 || { echo "pass 2 failed"; tail -5 $OUT/p2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob('gpurun_out/icpmc/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'dcm_mpc_cold' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v)/len(v):14.0f}  (dispatches {len(v)})")
PY
