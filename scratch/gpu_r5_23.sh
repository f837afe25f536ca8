#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 30 --warmup 5
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread
step benches 900 bash -c "python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3 && python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2 && python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2"
step prof_resnet 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_r5b -o prof --output-format csv -- python bench.py --steps 5 --warmup 2
