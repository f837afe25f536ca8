#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/host_overhead.py --steps 30 > gpurun_out/host_overhead.log 2>&1; rc=$?
head -3 gpurun_out/host_overhead.log; exit $rc
