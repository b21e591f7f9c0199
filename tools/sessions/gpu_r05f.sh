#!/bin/bash
# Round 5: the articulated-body solve in the floating-base kernels.  Their parity tests first
# (fb dynamics, closed loop, URDF, user systems), fbd_euler_kernel alone over one c5 period with
# and without it (BLF_FBD_ABA=0, two rounds), then the c5 bench line.  Stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05f}
timeout -k 10 500 python -u -m pytest tests/test_gpu_fb_dynamics.py tests/test_gpu_closed_loop.py tests/test_gpu_urdf.py tests/test_gpu_contact.py -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_fb.log 2>&1
rc=$?; grep -E "FAILED|ERROR|Error" gpurun_out/${T}_pytest_fb.log | head -5; tail -1 gpurun_out/${T}_pytest_fb.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for a in 1 0; do
    BLF_FBD_ABA=$a STREAM_TIME=1 timeout -k 10 200 python tools/stream_one.py fbd_euler > gpurun_out/${T}_fbd_aba${a}_$r.log 2>&1 || { echo "fbd aba=$a failed"; tail -3 gpurun_out/${T}_fbd_aba${a}_$r.log; exit 1; }
    echo -n "aba=$a round $r: "; grep median gpurun_out/${T}_fbd_aba${a}_$r.log
  done
done
for g in 2 1; do
  timeout -k 10 300 python bench.py --workload c5 --no-cpu --c5-groups $g > gpurun_out/${T}_c5_g$g.log 2>&1 || { echo "c5 g=$g failed"; tail -3 gpurun_out/${T}_c5_g$g.log; exit 1; }
  echo -n "c5 groups=$g: "; grep -v amdgpu.ids gpurun_out/${T}_c5_g$g.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['qp_status_counts'], d.get('base_height_range'))"
done
