#!/bin/bash
# Round 4: the closed-loop GPU tests (overlap bitwise among them), the hard c5 windows on the stamp
# build, then the c5 line without / with the overlap, two rounds.  Each GPU step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/bipedal-locomotion-framework_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_closed_loop.py tests/test_gpu_phased.py tests/test_gpu_c5_windows.py tests/test_abi.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04i_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04i_pytest.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
BLF_LIB=$L/libblf_stamps.so timeout -k 10 120 python tools/hard_windows_timing.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04i_hard_stamps.log || exit 1
for r in 1 2; do
  for o in 0 1; do
    timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-overlap $o > gpurun_out/r04i_c5_o${o}_$r.log 2>&1 || { echo "c5 o=$o failed"; exit 1; }
    echo -n "overlap=$o round $r: "; grep -v amdgpu.ids gpurun_out/r04i_c5_o${o}_$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'])"
  done
done
