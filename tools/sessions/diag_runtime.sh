#!/bin/bash
# Which HIP runtime does libblf.so bind to next to torch's, and does the init order matter?
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
{
echo "== ldd libblf.so"; ldd bipedal-locomotion-framework_amd/lib/libblf.so | grep -i "hip\|hsa\|rocm"
echo "== torch lib dir"; ls $(python -c "import torch,os;print(os.path.dirname(torch.__file__))")/lib | grep -i "amdhip\|hsa-runtime" 
echo "== env"; env | grep -i "HIP_\|ROCR\|HSA_\|CUDA_VISIBLE" 
echo "== order: torch first"
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'bipedal-locomotion-framework_amd')
import torch; print('torch avail', torch.cuda.is_available(), torch.cuda.device_count())
from blf import native
h = native.Handle(0); print('blf handle ok')
" 2>&1 | grep -v amdgpu.ids
echo "== order: blf first"
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'bipedal-locomotion-framework_amd')
from blf import native
h = native.Handle(0); print('blf handle ok')
import torch; print('torch avail', torch.cuda.is_available())
" 2>&1 | grep -v amdgpu.ids
echo "== in-process maps after torch init"
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'bipedal-locomotion-framework_amd')
import torch; torch.cuda.is_available()
from blf import native; native.lib()
print(''.join(l for l in open('/proc/self/maps') if 'amdhip' in l or 'hsa-runtime' in l))
" 2>&1 | grep -v amdgpu.ids | awk '{print \$6}' | sort -u
} > gpurun_out/diag_runtime.log 2>&1
cat gpurun_out/diag_runtime.log
