set -o pipefail
export TMPDIR=/tmp
# short-K dgrads with BN-backward sums: which tile family is fastest (the 256x256 pipelined tile holds one
# workgroup per CU; the 128-row tiles hold two or three)
out=gpurun_out/s47; mkdir -p $out
: > $out/probe.txt
for shp in "640 56 256 64 1 1" "640 28 512 128 1 1" "640 14 1024 256 1 1" "640 56 64 256 1 1"; do
  for env in "X=1" "PDA_GEMM_PP=0 PDA_GEMM_PP_CONV=0" "PDA_GEMM_PP=0 PDA_GEMM_PP_CONV=0 PDA_GEMM_WIDE=0" "PDA_GEMM_PP=0 PDA_GEMM_PP_CONV=0 PDA_GEMM_WIDE=0 PDA_GEMM_BIG=0"; do
    echo "## $env" >> $out/probe.txt
    env $env timeout -k 10 120 python -u tools/dgrad_bst_probe.py $shp 30 >> $out/probe.txt 2>&1 || exit 1
  done
done
cat $out/probe.txt
