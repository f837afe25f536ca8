set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s40; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -q -s --timeout 200 --timeout-method thread -k "fsdp_over_xgmi" > $out/t1.log 2>&1; echo "rc=$?"
grep -E "^\[rank|passed|failed" $out/t1.log | cut -c1-600
