# A/B of the transpose tile order as shipped (PNCX_XPOSE_ORDER unset = -1:
# diagonal for 2-D, row-major for merged, skewed for packed U strides just
# under a multiple of 2 MiB) against forced row-major (0) and diagonal (1).
#   bash tools/gpu_xpose_skew_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xauto_$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_imap.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAIL; tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
S="1024x1x260096 1024x1024x254 1024x1024x256 1024x1024x250 1000x1000x268 8192x1x8192 16384x1x4096 8192x1x8000"
for rep in 1 2; do
  for k in -1 0 1; do
    for d in put get; do
      PNCX_XPOSE_ORDER=$k PROBE_DIR=$d timeout -k 10 200 python3 $R/tools/transpose_probe.py $S > $O/k$k.$d.$rep.jsonl || { echo FAIL; exit 2; }
    done
  done
done
python3 - "$O" <<'PY'
import json, sys, glob
O = sys.argv[1]
res = {}
for f in sorted(glob.glob(O + "/k*.jsonl")):
    k = f.split("/")[-1].split(".")[0][1:]
    for l in open(f):
        r = json.loads(l)
        res.setdefault((r["shape"], r["dir"]), {}).setdefault(k, []).append(r["frac"])
for (sh, d), v in res.items():
    print(sh, d, " ".join(f"k{k}={v[k]}" for k in sorted(v, key=int)))
PY
