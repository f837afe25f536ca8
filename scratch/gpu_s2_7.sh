#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_7; mkdir -p $D
for cfg in "PDA_CONV_STEM_FWD=1" "PDA_CONV_STEM_FWD=0"; do
  env $cfg timeout -k 10 200 python tools/debug_stem_model.py > "$D/$cfg.log" 2>&1; rc=$?
  echo "== $cfg rc=$rc"; grep -v amdgpu.ids "$D/$cfg.log" | tail -4 | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
