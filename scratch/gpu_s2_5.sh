#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_5; mkdir -p $D
export TMPDIR=/tmp
T="tests/test_models_gpu.py::test_ddp_rccl_one_rank_group_matches_local tests/test_models_gpu.py::test_side_stream_wgrad_matches_single_stream"
for cfg in "X=1" "PDA_CONV_STEM_FWD=0" "PDA_CONV_STEM_WG=0" "PDA_CONV_STEM_FWD=0 PDA_CONV_STEM_WG=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest $T -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$D/t_${cfg// /_}.log" 2>&1
  rc=$?
  echo "== $cfg rc=$rc: $(grep -h 'passed\|failed' "$D/t_${cfg// /_}.log" | tail -1)"; grep -h "AssertionError" "$D/t_${cfg// /_}.log" | head -3
  if [ $rc -gt 1 ]; then exit $rc; fi
done
