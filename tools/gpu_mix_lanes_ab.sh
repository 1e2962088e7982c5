# A/B of the same-type batch kernel's block size (PNCX_MIX_BLOCK_LANES =
# 1024 (product) / 512 / 256) on C4, synchronous and asynchronous calls,
# alternating runs on one box; parity of the batch tests at 256 first.
#   bash tools/gpu_mix_lanes_ab.sh <tag> [rounds]
# (PNCX_MIX_BLOCK_LANES existed only in the A/B build; the product keeps 1024.)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/mix_ab_$1
mkdir -p $O
PNCX_MIX_BLOCK_LANES=256 timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q -k batch --timeout 120 --timeout-method thread > $O/parity256.txt 2>&1 || { echo PARITY_FAIL; tail -20 $O/parity256.txt; exit 1; }
tail -1 $O/parity256.txt
for i in $(seq 1 ${2:-3}); do
  for l in 1024 512 256; do
    for w in c4 c4_async; do
      t=${w}_$l.$i
      PNCX_MIX_BLOCK_LANES=$l timeout -k 10 120 python3 $R/bench.py --workload $w --no-cpu-baseline --steps 200 --warmup 20 > $O/$t.json 2> $O/$t.err || { echo FAIL $t; tail -5 $O/$t.err; exit 2; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], r['kernel_ms_avg'], r.get('call_ms_avg'), r['frac'], d['check_ok'])" $O/$t.json $t
    done
  done
done
