#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_xgmi.log; exit $rc
