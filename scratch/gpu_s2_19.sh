#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_19; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python tools/dgrad_phase_prof.py > $D/prof.log 2>&1; echo "rc=$?"
