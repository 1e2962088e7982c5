# A/B of the fused two-class batch launch on the C4 NC_ERANGE workload:
# two launches (PNCX_BATCH_FUSE=0) against the fused kernel with 1024- and
# 256-lane blocks (PNCX_FUSE_LANES), alternating runs on one box.
#   bash tools/gpu_fuse_ab.sh <tag> [rounds]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fuse_ab_$1
mkdir -p $O
for i in $(seq 1 ${2:-3}); do
  for v in "0 256" "1 1024" "1 256"; do
    set -- $v
    t=fuse$1_$2.$i
    PNCX_BATCH_FUSE=$1 PNCX_FUSE_LANES=$2 timeout -k 10 120 python3 $R/bench.py --workload c4_erange --no-cpu-baseline --steps 200 --warmup 20 > $O/$t.json 2> $O/$t.err || { echo FAIL $t; tail -5 $O/$t.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], r['kernel_ms_avg'], r.get('call_ms_avg'), r['frac'], d['check_ok'])" $O/$t.json $t
  done
done
