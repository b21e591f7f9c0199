#!/bin/bash
# Diagnostics: bench.py --workload c5 (closed loop, 16384 robots) with the product library and
# every lib/libblf_v*.so variant, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for lib in bipedal-locomotion-framework_amd/lib/libblf.so bipedal-locomotion-framework_amd/lib/libblf_v*.so; do
    BLF_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu 2>&1 \
        | grep -o '"ms_per_step": [0-9.]*' | sed "s|^|$(basename $lib) |" || exit 1
done
