# Skew factor scan on the two shapes whose packed U stride is 2^21 - 2^14 B:
# PNCX_XPOSE_ORDER = k for put and get, two alternating reps.
#   bash tools/gpu_xpose_kscan.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xk_$1
mkdir -p $O
S="1024x1x260096 1024x1024x254"
for rep in 1 2; do
  for k in 2 4 8 16 32 64 128; do
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
