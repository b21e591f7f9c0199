#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: 2 ranks over gloo sharing cuda:0
# (the driver's N>1 runs use RCCL, one rank per GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
BLF_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu \
    > gpurun_out/bench_2rank.log 2>&1
rc=$?
echo "2-rank rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_2rank.log | tail -5
exit $rc
