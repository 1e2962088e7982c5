# A/B of the per-XCD start offset of the varm transpose (PNCX_XPOSE_ROT),
# 2-D and 3-D shapes, both directions; the imap parity tests first.
#   bash tools/gpu_xpose_rot_ab.sh <tag>
# (PNCX_XPOSE_ROT existed only in the A/B build; the product has no rotation.)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xrot_$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_imap.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo TESTS_FAIL; tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
S="8192x1x8192 8192x1x8000 8192x1x8190 4096x1x16000 1024x1024x256 1024x1024x250 1000x1000x268 512x512x1000"
for rep in 1 2; do
  for rot in 0 1; do
    for d in put get; do
      PNCX_XPOSE_ROT=$rot PROBE_DIR=$d timeout -k 10 200 python3 $R/tools/transpose_probe.py $S > $O/rot$rot.$d.$rep.jsonl || { echo FAIL; exit 2; }
    done
  done
done
python3 - "$O" <<'PY'
import json, sys, glob
O = sys.argv[1]
res = {}
for f in sorted(glob.glob(O + "/rot*.jsonl")):
    rot = f.split("/")[-1][3]
    for l in open(f):
        r = json.loads(l)
        res.setdefault((r["shape"], r["dir"]), {}).setdefault(rot, []).append(r["frac"])
for (sh, d), v in res.items():
    print(sh, d, "rot0", v.get("0"), "rot1", v.get("1"))
PY
