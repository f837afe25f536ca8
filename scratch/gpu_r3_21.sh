#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_serving_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread -k batching > gpurun_out/eng.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/eng.log | tail -15; exit $rc
