set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "conv" > gpurun_out/s4/t.log 2>&1; rc=$?; tail -15 gpurun_out/s4/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_conv.py --batch 640 --iters 10 > gpurun_out/s4/conv_v2.jsonl 2>&1 || exit 1
PDA_CONV_WG3V2=0 timeout -k 10 400 python -u tools/bench_conv.py --batch 640 --iters 10 > gpurun_out/s4/conv_v1.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/s4/bench_v2.log 2>&1 && tail -1 gpurun_out/s4/bench_v2.log | cut -c1-200
PDA_CONV_WG3V2=0 timeout -k 10 300 python -u bench.py > gpurun_out/s4/bench_v1.log 2>&1 && tail -1 gpurun_out/s4/bench_v1.log | cut -c1-200
