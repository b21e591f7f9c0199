#!/bin/bash
# QP cold kernel A/B: FETCH_SIZE per dispatch (one --pmc pass per library) and kbench timing of
# the product library against each lib/libblf_v*.so variant.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for v in "" $(cd bipedal-locomotion-framework_amd/lib && ls libblf_v*.so 2>/dev/null | sed "s/libblf\(.*\)\.so/\1/"); do
  BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf$v.so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/pmc/f$v -o run -- python3 tools/kbench.py --reps 5 > gpurun_out/pmc/f$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import csv,glob,sys
f=glob.glob(f"gpurun_out/pmc/f{sys.argv[1]}/**/run_counter_collection.csv", recursive=True)[0]
v=[float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("dcm_mpc_cold")]
print(sys.argv[1] or "product", "FETCH_SIZE KiB per dispatch median", sorted(v)[len(v)//2], "x2 MB", 2*1024*sorted(v)[len(v)//2]/1e6)
PY
done
for r in 1 2 3; do KB_ARGS="--reps 30" bash tools/sessions/ab_multi.sh || exit 1; done
