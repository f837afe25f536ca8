set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/final4; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -2 $out/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py > $out/bench_default.log 2>&1 || { tail -20 $out/bench_default.log; exit 1; }
tail -1 $out/bench_default.log | cut -c1-400
timeout -k 10 300 python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3 > $out/gpt2.log 2>&1 || exit 1
tail -1 $out/gpt2.log | cut -c1-300
timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2 > $out/llama.log 2>&1 || exit 1
tail -1 $out/llama.log | cut -c1-300
