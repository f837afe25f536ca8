set -o pipefail
mkdir -p gpurun_out/s6
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "conv_fwd_dgrad_wgrad" > gpurun_out/s6/t.log 2>&1; rc=$?; tail -3 gpurun_out/s6/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_conv.py --batch 640 --iters 10 > gpurun_out/s6/conv_v2.jsonl 2>&1 || exit 1
PDA_CONV_WG3V2=0 timeout -k 10 400 python -u tools/bench_conv.py --batch 640 --iters 10 > gpurun_out/s6/conv_v1.jsonl 2>&1 || exit 1
