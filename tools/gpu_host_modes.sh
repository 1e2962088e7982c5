# Host-buffer conversion and file-level rates by stager mode (PNCX_HOST_ZC
# 0 copy / 1 zero-copy stores / 2 zero-copy both ways) and I/O threads:
# tools/host_roundtrip.py (4 GiB pncx_in_swapn / getn) and tools/file_bench.py.
#   bash tools/gpu_host_modes.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hm_$1
mkdir -p $O
for z in 0 1 2; do
  PNCX_HOST_ZC=$z timeout -k 10 200 python3 $R/tools/host_roundtrip.py --gib 2 > $O/rt_z$z.json 2> $O/rt_z$z.err || { echo FAIL rt $z; tail -5 $O/rt_z$z.err; exit 2; }
  echo "rt zc=$z $(tail -c 600 $O/rt_z$z.json)"
done
for z in 1 2; do
  for t in 1 8; do
    PNCX_HOST_ZC=$z PNCX_IO_THREADS=$t timeout -k 10 300 python3 $R/tools/file_bench.py --reps 3 > $O/fb_z$z.t$t.json 2> $O/fb_z$z.t$t.err || { echo FAIL fb $z $t; tail -5 $O/fb_z$z.t$t.err; exit 2; }
    echo "fb zc=$z io=$t $(tail -c 1500 $O/fb_z$z.t$t.json)"
  done
done
