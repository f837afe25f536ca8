#!/bin/bash
# checkpoint: full GPU test suite, smoke, bench (bs512 default), kernel profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_v23.txt 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_v23.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_v23.txt 2>&1 || exit 1
tail -1 gpurun_out/smoke_v23.txt
timeout -k 10 400 python bench.py > gpurun_out/bench_v23.json 2>gpurun_out/bench_v23.err || exit 1
cat gpurun_out/bench_v23.json | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof43 -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof43.log 2>&1 || exit 1
echo ok
