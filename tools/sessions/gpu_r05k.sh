#!/bin/bash
# Quintic evaluation A/B: product vs lib/libblf_vq_*.so (no spline staging, plain stores, direct
# per-lane stores), twice each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for r in 1 2; do STREAM_KERNEL=quintic bash tools/sessions/ab_stream.sh || exit 1; done
