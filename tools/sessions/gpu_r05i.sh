#!/bin/bash
# A/B of the contact-law branch in the fbd kernels on the c5 bench: product library vs
# lib/libblf_nolaw.so (-DBLF_FBD_LAWS=0), alternating, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$PWD/bipedal-locomotion-framework_amd/lib/libblf_nolaw.so
for r in 1 2; do
  for lib in base nolaw; do
    if [ $lib = base ]; then unset BLF_LIB; else export BLF_LIB=$V; fi
    timeout -k 10 300 python bench.py --workload c5 --no-cpu > gpurun_out/r05i_${lib}_$r.log 2>&1 || { echo "$lib failed"; tail -3 gpurun_out/r05i_${lib}_$r.log; exit 1; }
    echo -n "$lib $r: "; grep -v amdgpu.ids gpurun_out/r05i_${lib}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])"
  done
done
