#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_kern 600 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider -k "batchnorm or conv"
step bench 300 python bench.py --steps 20 --warmup 5
step xgmi 200 python -m pytest tests/test_xgmi_gpu.py -q -x -p no:cacheprovider
for op in fwd wgrad; do
  step pmc_$op 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_$op -o p -- python tools/conv_one.py $op 14 256 256 3 1 5
  step pmc2_$op 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/pmc2_$op -o p -- python tools/conv_one.py $op 14 256 256 3 1 5
done
