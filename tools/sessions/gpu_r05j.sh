#!/bin/bash
# Round 5: the hull's edge-difference triple test and the unpadded slab store (quintic, fbk):
# kernel / staging / contact GPU tests, the stream roofline lines (event timing), then the
# contact-law A/B on c5 (tools/sessions/gpu_r05i.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05j}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_staging.py tests/test_gpu_contact.py tests/test_gpu_phase_expand.py -v -x -m gpu --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${T}_pytest_gpu.log | head -20; tail -1 gpurun_out/${T}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stream_bench.py --out gpurun_out/${T}_stream.json > gpurun_out/${T}_stream.log 2>&1 || { tail -5 gpurun_out/${T}_stream.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_stream.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print('%-28s %.4f ms  %.0f GB/s  frac %.3f' % (d['kernel'], d['ms'], d['achieved_gbs'], d['frac']))"
bash tools/sessions/gpu_r05i.sh
