set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
hipcc -O3 --offload-arch=gfx950 -Wno-unused-value -o /tmp/ubench_dpp tools/ubench_dpp.hip && timeout -k 10 60 /tmp/ubench_dpp
bash tools/sessions/gpu_session.sh
