#!/bin/bash
# First GPU pass: kernel numerics tests, short bench, rocprofv3 kernel stats of the bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench1.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
