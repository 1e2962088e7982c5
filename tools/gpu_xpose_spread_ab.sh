# Transpose tile order: the shipped order (skew 8 put / 32 get for the
# x254 stride, row-major merged, diagonal 2-D) against "spread"
# (PNCX_XPOSE_ORDER=2000: p tiles run (tp * ~tp/64) mod tp, so the tiles
# resident at once cover the packed address bits below the column stride);
# whole processes alternating, 2 rounds (tools/transpose_probe.py)
# (historical: the knob it A/Bs was removed after the run; kept as the record of how its profiles/ file was made)
set -o pipefail
O=${OUT:-gpurun_out/r06i_xpose_spread_ab.txt}
mkdir -p gpurun_out
: > $O
for r in 1 2; do
  for dir in put get; do
    for ord in -1 2000 2000 -1; do
      echo "round $r dir $dir order $ord" >> $O
      PROBE_DIR=$dir PNCX_XPOSE_ORDER=$ord timeout -k 10 200 python3 tools/transpose_probe.py 1024x1024x254 1024x1024x256 1024x1024x250 >> $O 2>&1 || exit 1
    done
  done
done
