# A/B of the transpose tile shape (PNCX_XPOSE_TILE 0: 64 (P) x 128 (U),
# 1: 128 x 64) on the merged 3-D shapes and the 2-D ones, both directions,
# alternating; the imap parity tests with the tall tiles first.
#   bash tools/gpu_xpose_tile_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xtile_$1
mkdir -p $O
PNCX_XPOSE_TILE=1 timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_imap.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_tall.txt 2>&1 || { echo TESTS_FAIL; tail -20 $O/tests_tall.txt; exit 1; }
tail -1 $O/tests_tall.txt
S="1024x1024x254 1024x1024x256 1024x1024x250 1000x1000x268 512x512x1000 8192x1x8192 1024x1x260096"
for rep in 1 2; do
  for t in 0 1; do
    for d in put get; do
      PNCX_XPOSE_TILE=$t PROBE_DIR=$d timeout -k 10 200 python3 $R/tools/transpose_probe.py $S > $O/t$t.$d.$rep.jsonl || { echo FAIL; exit 2; }
    done
  done
done
python3 - "$O" <<'PY'
import json, sys, glob
O = sys.argv[1]
res = {}
for f in sorted(glob.glob(O + "/t*.jsonl")):
    t = f.split("/")[-1][1]
    for l in open(f):
        r = json.loads(l)
        res.setdefault((r["shape"], r["dir"]), {}).setdefault(t, []).append(r["frac"])
for (sh, d), v in res.items():
    print(sh, d, "64x128", v.get("0"), "128x64", v.get("1"))
PY
