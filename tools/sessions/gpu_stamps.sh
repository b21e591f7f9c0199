set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_stamps.so timeout -k 10 200 python tools/kbench.py > gpurun_out/kb_stamps.log 2>&1 || exit $?
cat gpurun_out/kb_stamps.log
