#!/bin/bash
cd "$GRAFT_REPO_ROOT/tools" || exit 1
mkdir -p ../gpurun_out
timeout -k 10 200 python bench_w8_splits.py > ../gpurun_out/w8_splits.log 2>&1; rc=$?; grep -v amdgpu ../gpurun_out/w8_splits.log; exit $rc
