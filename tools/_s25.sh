set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s25; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.txt 2>&1; rc=$?
tail -5 $out/pytest_gpu.txt
exit $rc
