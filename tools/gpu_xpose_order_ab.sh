# A/B of the transpose tile order (PNCX_XPOSE_ORDER 0 row-major / 1
# diagonal), 2-D and 3-D shapes, both directions, alternating; the imap
# parity tests first.
#   bash tools/gpu_xpose_order_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xord_$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_imap.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAIL; tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
S="8192x1x8192 8192x1x8000 4096x1x16000 16384x1x4096 1024x1024x256 1024x1024x254 1024x1024x250 1000x1000x268 512x512x1000"
for rep in 1 2; do
  for ord in 0 1; do
    for d in put get; do
      PNCX_XPOSE_ORDER=$ord PROBE_DIR=$d timeout -k 10 200 python3 $R/tools/transpose_probe.py $S > $O/ord$ord.$d.$rep.jsonl || { echo FAIL; exit 2; }
    done
  done
done
python3 - "$O" <<'PY'
import json, sys, glob
O = sys.argv[1]
res = {}
for f in sorted(glob.glob(O + "/ord*.jsonl")):
    o = f.split("/")[-1][3]
    for l in open(f):
        r = json.loads(l)
        res.setdefault((r["shape"], r["dir"]), {}).setdefault(o, []).append(r["frac"])
for (sh, d), v in res.items():
    print(sh, d, "rowmajor", v.get("0"), "diagonal", v.get("1"))
PY
