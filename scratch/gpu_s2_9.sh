#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_9; mkdir -p $D
export PDA_CONV_STEM_FWD=1 PDA_BN_STAT_ROWS=256
timeout -k 10 300 python -u -m pytest "tests/test_models_gpu.py::test_ddp_rccl_one_rank_group_matches_local" -q -p no:cacheprovider --timeout 200 --timeout-method thread > $D/ddp_rows256.log 2>&1
echo "== ddp stat rows 256 rc=$?: $(grep -h 'passed\|failed' $D/ddp_rows256.log | tail -1)"; grep -h "AssertionError" $D/ddp_rows256.log | head -3
