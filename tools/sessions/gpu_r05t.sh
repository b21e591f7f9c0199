#!/bin/bash
# A/B of the fp32 search's hand-over threshold (N / BLF_HANDOVER_DIV knots changed): product (16)
# vs lib/libblf_vho{8,32,1000}.so on the configs[1] bench, two alternating rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 16 8 32 1000; do
    if [ $v = 16 ]; then unset BLF_LIB; else export BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_vho$v.so; fi
    timeout -k 10 300 python bench.py --no-cpu --steps 50 > gpurun_out/r05t_${v}_$r.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r05t_${v}_$r.log; exit 1; }
    echo -n "div $v round $r: "; grep -v amdgpu.ids gpurun_out/r05t_${v}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
