# Is the merged 1024 x 1024 x 254 transpose slow because of its packed column
# stride (2^21 - 2^14 bytes)?  The same stride in a 2-D transpose
# (1024 x 260096 doubles) against 2^21 (1024 x 262144) and 2^21 - 3*2^14
# (1024 x 256000), both tile orders, both directions.
#   bash tools/gpu_xpose_stride.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xstr_$1
mkdir -p $O
S="1024x1x260096 1024x1x262144 1024x1x256000 1024x1024x254 1024x1024x256"
for ord in 0 1; do
  for d in put get; do
    PNCX_XPOSE_ORDER=$ord PROBE_DIR=$d timeout -k 10 200 python3 $R/tools/transpose_probe.py $S > $O/ord$ord.$d.jsonl || { echo FAIL; exit 2; }
  done
done
for f in $O/ord*.jsonl; do echo "# $(basename $f)"; cat $f; done
