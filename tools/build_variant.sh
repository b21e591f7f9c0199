#!/bin/bash
# Diagnostics: build the working copy of one kernel source (VSRC, default dcm_mpc_ipm; plus extra
# hipcc flags) into lib/libblf_<name>.so next to the product library, for A/B runs with
# tools/sessions/ab_multi.sh.
#   [VSRC=dcm_mpc_as] tools/build_variant.sh <name> [hipcc flags...]
set -eu
cd "$(dirname "$0")/../bipedal-locomotion-framework_amd"
src=${VSRC:-dcm_mpc_ipm}
name=$1; shift
# the product builds the QP and floating-base kernels with the iterative-ILP scheduler (Makefile QPSCHED)
{ [ "$src" = dcm_mpc_as ] || [ "$src" = fb_dynamics ]; } && set -- -mllvm -amdgpu-sched-strategy=iterative-ilp "$@"
mkdir -p build/variant_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
    -I../include -Icsrc "$@" -c csrc/$src.hip -o build/variant_$name/$src.o
objs=$(ls build/*.o | grep -v "/$src.o\$" | grep -v '/host_')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libblf_$name.so build/variant_$name/$src.o $objs
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
    -I../include -Icsrc "$@" -c csrc/$src.hip -o /tmp/variant_$name.devonly.o --cuda-device-only \
    -Rpass-analysis=kernel-resource-usage 2>&1 | grep -i "VGPRs:\|Scratch\|Occupancy" | sort | uniq -c \
    | sed "s/.*remark: */$name: /" || true
