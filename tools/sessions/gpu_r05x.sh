#!/bin/bash
# Round 5 A/B: the IPM kernel's 16-slot loops without the early exit (the knot record stays in
# registers instead of 424 B of scratch), lib/libblf_v16.so, against the product: mc (cold window
# stage 2) and c2; then the GPU suite on the variant.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
P=bipedal-locomotion-framework_amd/lib
for round in 1 2; do
  for lib in libblf.so libblf_v16.so; do
    BLF_LIB=$PWD/$P/$lib timeout -k 10 200 python bench.py --workload mc --steps 20 --warmup 3 --no-cpu > gpurun_out/r05x_mc_${lib}_$round.log 2>&1 || exit 1
    echo "mc $lib $round $(grep -o '"ms_per_step": [0-9.]*\|"warm_ms[a-z_]*": [0-9.]*' gpurun_out/r05x_mc_${lib}_$round.log | tr '\n' ' ')"
    BLF_LIB=$PWD/$P/$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/r05x_c2_${lib}_$round.log 2>&1 || exit 1
    echo "c2 $lib $round $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r05x_c2_${lib}_$round.log)"
  done
done
BLF_LIB=$PWD/$P/libblf_v16.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05x_pytest_v16.log 2>&1; tail -3 gpurun_out/r05x_pytest_v16.log
