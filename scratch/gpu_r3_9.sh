#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/debug_w8_model.py > gpurun_out/dbg_w8.log 2>&1; echo rc=$?; cat gpurun_out/dbg_w8.log | grep -v amdgpu | head -60
