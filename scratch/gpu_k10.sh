#!/bin/bash
# native comm (default priority, pooled events) vs c10d vs no comm; GPT-2 copy sites + kernel table;
# PP x DP rehearsal over gloo (4 ranks on one GPU)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k10
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/k10/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/k10/$name.log | grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|UserWarning\|default_pg" | tail -12 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step comm_tests 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_models_gpu.py -k "rccl"
for r in 1 2; do
  step native_$r 200 python bench.py --steps 20 --warmup 5
  step c10d_$r 200 env PDA_COMM=c10d python bench.py --steps 20 --warmup 5
  step nocomm_$r 200 env PDA_DDP_FORCE_COMM=0 python bench.py --steps 20 --warmup 5
done
step copies 300 python tools/find_copies.py --model gpt2 --steps 2 --batch 8
step prof_gpt2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/k10/prof_gpt2 -o p --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 2
step ppdp_gloo 400 env PDA_DIST_BACKEND=gloo python -m pytorchdistributed_amd.bench.gpt2xl_pp --gpus 4 --pp 2 --layers 8 --micro 4 --micro-batch 2 --steps 3 --warmup 1
