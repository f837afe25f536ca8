#!/bin/bash
# direct-epilogue equality + A/B; transformer benches after this round's FSDP / pipeline / communicator
# changes; smoke; kernel traces of the headline step (native communicator vs ProcessGroupNCCL)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k11
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/k11/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/k11/$name.log | grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl\|UserWarning\|default_pg\|^W2026\|^E2026" | tail -6 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step epi_test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "direct_epilogue or conv_fwd_epilogue or masked_addend"
for r in 1 2; do
  step staged_$r 200 python bench.py --steps 20 --warmup 5
  step direct_$r 200 env PDA_WIDE_EPI_DIRECT=1 python bench.py --steps 20 --warmup 5
done
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step llama_fsdp 400 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step gpt2xl_pp 300 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2
step trace_native 200 rocprofv3 --kernel-trace --stats -d gpurun_out/k11/tr_native -o p --output-format csv -- python bench.py --steps 6 --warmup 3
step trace_c10d 200 env PDA_COMM=c10d rocprofv3 --kernel-trace --stats -d gpurun_out/k11/tr_c10d -o p --output-format csv -- python bench.py --steps 6 --warmup 3
