#!/bin/bash
# Round 3, late: compiler scheduling strategies of the QP kernels (lib/libblf_vs*.so: max-ilp,
# iterative-ilp, metric bias 0) against the product on kbench (B = 1 N = 50, B = 4096, 65 536),
# alternating, two rounds; then the 2-rank gloo rehearsal of the bench on one GPU (c2 and c5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
: > gpurun_out/sched_ab.log
for r in 1 2; do
  for lib in libblf libblf_vs1 libblf_vs2 libblf_vs3; do
    for cfg in "--batch 1 --horizon 50 --reps 200" "--batch 4096 --horizon 100 --reps 50" "--batch 65536 --horizon 100 --reps 10"; do
      BLF_LIB=$L/$lib.so timeout -k 10 120 python tools/kbench.py $cfg 2>&1 | grep -v amdgpu.ids >> gpurun_out/sched_ab.log || exit 1
    done
  done
done
cat gpurun_out/sched_ab.log
bash tools/sessions/gpu_multirank.sh || exit 1
BLF_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --workload c5 --steps 3 --warmup 1 --no-cpu \
    > gpurun_out/bench_2rank_c5.log 2>&1 || { echo "c5 2-rank failed"; tail -5 gpurun_out/bench_2rank_c5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_2rank_c5.log | tail -1 | cut -c1-300
