#!/bin/bash
# Build the extension from a given git revision into gpurun_ab/<name>/ (a full package copy), so an
# A/B benchmark can import both builds on the same GPU box:  PYTHONPATH=gpurun_ab/<name> python ...
# usage: tools/ab_build.sh <rev> <name>
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" worktree add -f --detach "$tmp" "$rev" >/dev/null
(cd "$tmp" && python -c "import pytorchdistributed_amd._build as b; b.build()" >/dev/null)
rm -rf "$root/gpurun_ab/$name" && mkdir -p "$root/gpurun_ab/$name"
cp -r "$tmp/pytorchdistributed_amd" "$root/gpurun_ab/$name/"
git -C "$root" worktree remove --force "$tmp"
echo "built $rev into gpurun_ab/$name"
