#!/bin/bash
# Diagnostics: build the working copy of csrc/dcm_mpc_ipm.hip (plus extra hipcc flags) into
# lib/libblf_<name>.so next to the product library, for A/B runs with tools/ab_multi.sh.
#   tools/build_variant.sh <name> [hipcc flags...]
set -eu
cd "$(dirname "$0")/../bipedal-locomotion-framework_amd"
name=$1; shift
mkdir -p build/variant_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
    -I../include -Icsrc "$@" -c csrc/dcm_mpc_ipm.hip -o build/variant_$name/dcm_mpc_ipm.o
objs=$(ls build/*.o | grep -v '/dcm_mpc_ipm.o$' | grep -v '/host_')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libblf_$name.so build/variant_$name/dcm_mpc_ipm.o $objs
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
    -I../include -Icsrc "$@" -c csrc/dcm_mpc_ipm.hip -o /tmp/variant_$name.devonly.o --cuda-device-only \
    -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A12 "Function Name: .*ILi128ELb0ELb0" \
    | grep -i "VGPRs:\|Spill" | sed "s/.*remark: */$name: /" || true
