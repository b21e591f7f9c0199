#!/bin/bash
# Diagnostics: resource usage (VGPRs, spills, scratch, occupancy) of the kernels of one source
# whose mangled name matches a pattern.   tools/kres.sh <src> <pattern> [hipcc flags...]
cd "$(dirname "$0")/../bipedal-locomotion-framework_amd"
src=$1; pat=$2; shift 2
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -I../include -Icsrc \
    --cuda-device-only -c csrc/$src.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
    sed 's/.*remark: *//;s/ \[-Rpass.*//' | awk -v pat="$pat" '
      /Function Name:/ {show = ($0 ~ pat); if (show) {n=$3; sub(/^_ZN3blf12_GLOBAL__N_1[0-9]+/, "", n); printf "%s:", substr(n,1,60)}}
      show && /VGPRs:|AGPRs:|VGPRs Spill|ScratchSize|Occupancy|LDS Size/ {printf " %s", $0}
      show && /LDS Size/ {print ""}'
