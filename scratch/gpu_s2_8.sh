#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_8; mkdir -p $D
export PDA_CONV_STEM_FWD=1
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py::test_side_stream_wgrad_matches_single_stream -q -p no:cacheprovider --timeout 200 --timeout-method thread > $D/side_only.log 2>&1
echo "== side only rc=$?: $(grep -h 'passed\|failed' $D/side_only.log | tail -1)"; grep -h "AssertionError" $D/side_only.log | head -2
timeout -k 10 300 python -u -m pytest "tests/test_models_gpu.py::test_ddp_rccl_one_rank_group_matches_local" -q -p no:cacheprovider --timeout 200 --timeout-method thread > $D/ddp.log 2>&1
echo "== ddp rc=$?: $(grep -h 'passed\|failed' $D/ddp.log | tail -1)"; grep -h "AssertionError" $D/ddp.log | head -3
