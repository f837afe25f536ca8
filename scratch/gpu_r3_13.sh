#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ulysses_gpu.py -v -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ulysses.log 2>&1; rc=$?; tail -15 gpurun_out/ulysses.log; exit $rc
