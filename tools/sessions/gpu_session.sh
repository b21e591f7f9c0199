set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 480 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/kbench.py > gpurun_out/kb_default.log 2>&1 || exit $?
cat gpurun_out/kb_default.log
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_variant.so timeout -k 10 200 python tools/kbench.py > gpurun_out/kb_w3.log 2>&1 || exit $?
cat gpurun_out/kb_w3.log
BLF_LIB=$PWD/bipedal-locomotion-framework_amd/lib/libblf_stamps.so timeout -k 10 200 python tools/kbench.py > gpurun_out/kb_stamps.log 2>&1 || exit $?
cat gpurun_out/kb_stamps.log
