#!/bin/bash
# LDS / VALU pressure counters of the QP kernel (kbench, B=4096), one rocprofv3 --pmc pass per set.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/ldspmc
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
grep -o "SQ_[A-Z0-9_]*" $OUT/avail.txt | sort -u > $OUT/sq_names.txt
KB="tools/kbench.py --reps 5 --batch ${KB_BATCH:-4096}"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM"; do
    i=$((i+1))
    ok=1; for c in $set; do grep -qx $c $OUT/sq_names.txt || { echo "missing $c"; ok=0; }; done
    s2=$(for c in $set; do grep -qx $c $OUT/sq_names.txt && echo -n "$c "; done)
    timeout -s KILL 90 rocprofv3 --pmc $s2 -T --output-format csv -d $OUT/p$i -o run -- python3 $KB > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob('gpurun_out/ldspmc/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'dcm_mpc_as' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v)/len(v):14.0f}  (dispatches {len(v)})")
PY
