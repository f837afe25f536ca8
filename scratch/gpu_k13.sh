#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k13
export TMPDIR=/tmp
timeout -k 10 400 python tools/conv_batch_scaling.py > gpurun_out/k13/scaling.log 2>&1
rc=$?; echo "== scaling rc=$rc"; grep "^{" gpurun_out/k13/scaling.log | cut -c1-900
exit $rc
