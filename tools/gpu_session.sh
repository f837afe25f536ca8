#!/bin/bash
# One GPU-box session: named steps, each under its own time limit; a crash-class exit (timeout, abort,
# segfault) ends the session, a plain failure (tests failing, exit 1) is logged and the next step runs.
#   bash tools/gpu_session.sh OUTDIR STEP [STEP ...]      (steps: see the case below)
out=$1; shift
mkdir -p "$out"
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[session] $name: $*"
  timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "[session] $name exit=$rc"
  tail -3 "$out/$name.log"
  case $rc in 124|134|137|139) echo "[session] stopping after $name (exit $rc)"; exit $rc;; esac
  return 0
}
for step in "$@"; do
  case $step in
    gemm_tests) run gemm_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or conv" ;;
    gpu_tests) run gpu_tests 1050 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    lab) run lab 400 python -u tools/gemm_lab.py --variants 2,6,10,100 --layouts nt,tn --no-native --shapes 4096x4096x4096,8192x8192x8192,32768x3072x1024,32768x1024x4096,16384x4096x4096 ;;
    resnet_ab) run resnet_ab 900 bash tools/ab_env.sh "$out/resnet_ab.jsonl" 2 "PDA_GEMM_PP=1" "PDA_GEMM_PP=0" -- python -u bench.py --steps 20 --warmup 5 ;;
    gpt2_ab) run gpt2_ab 900 bash tools/ab_env.sh "$out/gpt2_ab.jsonl" 1 "PDA_MLP_FUSED=1" "PDA_MLP_FUSED=0" -- python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 8 --warmup 3 ;;
    bench) run bench 600 python -u bench.py ;;
    conv_table) run conv_table 600 python -u tools/bench_conv.py --batch 640 --iters 10 ;;
    gpt2) run gpt2 300 python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 8 --warmup 3 ;;
    llama) run llama 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 ;;
    lab4) run lab4 400 python -u tools/gemm_lab.py --variants 2,200 --layouts nt,nn,tn --shapes 4096x4096x4096,8192x8192x8192,32768x3072x1024,32768x1024x4096,16384x4096x4096,16384x28672x4096 ;;
    gpt2_prof) export TMPDIR=/tmp; run gpt2_prof 600 rocprofv3 --kernel-trace --output-format csv -d "$out/gpt2_prof" -o run -- python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 2 ;;
    llama_prof) export TMPDIR=/tmp; run llama_prof 600 rocprofv3 --kernel-trace --output-format csv -d "$out/llama_prof" -o run -- python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 2 --warmup 2 ;;
    resnet_prof) export TMPDIR=/tmp; PDA_WGRAD_STREAM=0 run resnet_prof 600 rocprofv3 --kernel-trace --output-format csv -d "$out/resnet_prof" -o run -- python -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 3 --warmup 3 ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    # multi-rank rehearsal on a one-GPU box: ranks share the GPU over gloo (RCCL refuses two ranks per
    # device), so the DDP and pipeline x DDP paths run with world > 1 on the native kernels
    rehearse_dp) PDA_DIST_BACKEND=gloo run rehearse_dp2 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --batch 256
                 PDA_DIST_BACKEND=gloo run rehearse_dp4 300 python -u bench.py --gpus 4 --steps 5 --warmup 2 --batch 128 ;;
    rehearse_pp) PDA_DIST_BACKEND=gloo run rehearse_pp 400 python -u -m pytorchdistributed_amd.bench.gpt2xl_pp --gpus 4 --pp 2 --micro 4 --micro-batch 4 --steps 3 --warmup 1 ;;
    gpt2xl_pp) run gpt2xl_pp 600 python -u -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 4 --warmup 2 ;;
    gpt2xl_pp_il) run gpt2xl_pp_il 600 python -u -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 4 --warmup 2 --schedule interleaved --chunks 2 ;;
    llama_forced) PDA_FSDP_FORCE_COMM=1 run llama_forced 500 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 ;;
    bench20) run bench20 300 python -u bench.py --steps 20 --warmup 5 ;;
    *) echo "[session] unknown step $step" ;;
  esac
done
