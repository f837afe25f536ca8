set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s20; mkdir -p $out
timeout -k 10 500 python -u tools/op_attrib.py pytorchdistributed_amd.bench.llama_fsdp --steps 2 --warmup 1 > $out/ll_ops.log 2>&1 || { tail -20 $out/ll_ops.log; exit 1; }
grep -v "^{" $out/ll_ops.log | grep -v "amdgpu.ids" | head -40
