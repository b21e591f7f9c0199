#!/bin/bash
# Round 5 A/B: the warm kernel's cold re-solve of the QPs its passes do not certify
# (BLF_WARM_RETRY=1, lib/libblf_vwr.so) against the product library: c5 closed loop (alternating,
# twice each), receding horizon, three-contact warm.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
P=bipedal-locomotion-framework_amd/lib
for round in 1 2; do
  for lib in libblf.so libblf_vwr.so; do
    BLF_LIB=$PWD/$P/$lib timeout -k 10 200 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/r05v_c5_${lib}_$round.log 2>&1 || exit 1
    echo "c5 $lib $round $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05v_c5_${lib}_$round.log) $(grep -o '"solved": [0-9]*\|"max_iter": [0-9]*' gpurun_out/r05v_c5_${lib}_$round.log | tr '\n' ' ')"
  done
done
for lib in libblf.so libblf_vwr.so; do
  for w in rh mc; do
    BLF_LIB=$PWD/$P/$lib timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > gpurun_out/r05v_${w}_${lib}.log 2>&1 || exit 1
    echo "$w $lib $(grep -o '"ms_per_step": [0-9.]*\|"warm_ms[a-z_]*": [0-9.]*' gpurun_out/r05v_${w}_${lib}.log | tr '\n' ' ')"
  done
done
