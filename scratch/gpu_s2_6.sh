#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s2_6
timeout -k 10 300 python tools/stem_debug.py > gpurun_out/s2_6/stem_debug.log 2>&1; rc=$?; cat gpurun_out/s2_6/stem_debug.log | tail -8; exit $rc
