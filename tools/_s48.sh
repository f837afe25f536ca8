set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s48; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -v --timeout 300 --timeout-method thread -k "parameter_server or rccl" > $out/t.log 2>&1 || { tail -40 $out/t.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $out/t.log | tail -12
