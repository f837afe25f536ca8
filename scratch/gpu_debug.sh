cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scratch/debug_resnet.py > gpurun_out/debug.log 2>&1; echo rc=$?
cat gpurun_out/debug.log | grep -v amdgpu.ids
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -15 gpurun_out/pytest_gpu.log
