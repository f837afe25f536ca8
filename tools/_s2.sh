set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "bwd_stats or resnet50_native" > gpurun_out/s2/t.log 2>&1; rc=$?; tail -15 gpurun_out/s2/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/s2/bench_on.log 2>&1 && tail -1 gpurun_out/s2/bench_on.log
PDA_BN_BWD_EPILOGUE=0 timeout -k 10 300 python -u bench.py > gpurun_out/s2/bench_off.log 2>&1 && tail -1 gpurun_out/s2/bench_off.log
timeout -k 10 300 python -u bench.py > gpurun_out/s2/bench_on2.log 2>&1 && tail -1 gpurun_out/s2/bench_on2.log
