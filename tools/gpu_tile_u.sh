# A/B of tiles per block for the direct-shape conversion kernels
# (PNCX_TILE_U = 1, 2, 4) on a list of pairs, plus parity at U = 2 and 4.
#   bash tools/gpu_tile_u.sh <tag> <pairs>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tile_u_$1
mkdir -p $O
for u in 2 4; do
  PNCX_TILE_U=$u timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_all_kinds.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/parity_u$u.txt 2>&1 || { echo PARITY_FAIL $u; tail -20 $O/parity_u$u.txt; exit 1; }
  tail -1 $O/parity_u$u.txt
done
for rep in 1 2; do
  for u in 1 2 4; do
    PNCX_TILE_U=$u timeout -k 10 200 python3 $R/tools/matrix_bench.py --pairs $2 --reps 5 > $O/u$u.$rep.jsonl || { echo BENCH_FAIL $u; exit 2; }
    python3 -c "
import json,sys
for l in open(sys.argv[1]):
    r=json.loads(l); print('u=$u rep=$rep', r['dir'], r['xtype'], r['itype'], r['frac'])" $O/u$u.$rep.jsonl
  done
done
