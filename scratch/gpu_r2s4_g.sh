#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step dualtest 200 python -u -m pytest tests/test_kernels_gpu.py -k "dual_bn or stem_bn" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step models 400 python -u -m pytest tests/test_models_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
CFGS="${CFGS:-X=1;PDA_DUAL_BN=0}" bash scratch/gpu_r2s4_d.sh
