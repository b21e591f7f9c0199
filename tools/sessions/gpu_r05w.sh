#!/bin/bash
# Round 5: GPU suite with the warm kernel's cold re-solve (product, BLF_WARM_RETRY=1), then the A/B
# against it off (lib/libblf_v0.so): c5 (alternating, three times each), receding horizon, three-contact warm.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05w_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05w_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r05w_pytest_gpu.log
P=bipedal-locomotion-framework_amd/lib
for round in 1 2 3; do
  for lib in libblf.so libblf_v0.so; do
    BLF_LIB=$PWD/$P/$lib timeout -k 10 200 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/r05w_c5_${lib}_$round.log 2>&1 || exit 1
    echo "c5 $lib $round $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05w_c5_${lib}_$round.log) $(grep -o '"solved": [0-9]*\|"max_iter": [0-9]*' gpurun_out/r05w_c5_${lib}_$round.log | tr '\n' ' ')"
  done
done
for round in 1 2; do
for lib in libblf.so libblf_v0.so; do
  for w in rh mc; do
    BLF_LIB=$PWD/$P/$lib timeout -k 10 200 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > gpurun_out/r05w_${w}_${lib}_$round.log 2>&1 || exit 1
    echo "$w $lib $round $(grep -o '"ms_per_step": [0-9.]*\|"warm_ms[a-z_]*": [0-9.]*' gpurun_out/r05w_${w}_${lib}_$round.log | tr '\n' ' ')"
  done
done
done
