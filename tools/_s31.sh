set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s31; mkdir -p $out
for shape in "640 56 128 128 3 2" "640 28 256 256 3 2" "640 14 512 512 3 2" "640 56 64 64 3 1" "640 28 128 128 3 1" "640 56 256 64 1 1" "640 56 64 256 1 1"; do
  timeout -k 10 120 python -u tools/dgrad_bst_probe.py $shape > $out/p.log 2>&1 || { cat $out/p.log; exit 1; }
  grep -v amdgpu $out/p.log
done
