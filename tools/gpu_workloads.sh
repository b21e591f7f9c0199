set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload c3 --steps 5 --warmup 1 > gpurun_out/bench_c3.log 2>&1; echo "c3 rc=$?"; tail -2 gpurun_out/bench_c3.log
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2>&1; echo "c5 rc=$?"; tail -2 gpurun_out/bench_c5.log
