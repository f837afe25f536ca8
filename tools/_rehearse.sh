set -o pipefail
export TMPDIR=/tmp
# multi-rank rehearsal of the final tree on a one-GPU box: ranks share the GPU over gloo (RCCL refuses
# two ranks per device), so the DDP / pipeline x DDP paths run with world > 1 on the native kernels
out=gpurun_out/rehearse; mkdir -p $out
export PDA_DIST_BACKEND=gloo
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --batch 256 > $out/rn2.log 2>&1 || { tail -30 $out/rn2.log; exit 1; }
tail -1 $out/rn2.log
timeout -k 10 300 python -u bench.py --gpus 4 --steps 5 --warmup 2 --batch 128 > $out/rn4.log 2>&1 || { tail -30 $out/rn4.log; exit 1; }
tail -1 $out/rn4.log
timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.gpt2xl_pp --gpus 4 --pp 2 --micro 4 --micro-batch 4 --steps 3 --warmup 1 > $out/pp.log 2>&1 || { tail -30 $out/pp.log; exit 1; }
tail -1 $out/pp.log
