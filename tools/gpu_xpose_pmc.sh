# rocprofv3 counters of the varm transpose (k_imap_tile, put) for
# 8192 x 8192 doubles in row-major and diagonal tile order and for the
# merged 3-D shapes 1024 x 1024 x 254 / x 256: one pass per counter group,
# each under its own limit (tools/transpose_probe.py, 70 launches a shape).
#   bash tools/gpu_xpose_pmc.sh <tag> [counter groups...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/xpmc_$1
shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
for spec in "0:8192x1x8192" "1:8192x1x8192" "0:1024x1024x254" "0:1024x1024x256" "1:1024x1024x254"; do
  ord=${spec%%:*}; sh=${spec#*:}
  i=0
  for grp in "$@"; do
    i=$((i+1))
    PNCX_XPOSE_ORDER=$ord timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/o${ord}_${sh}_$i -o p -- python3 $R/tools/transpose_probe.py $sh > $O/o${ord}_${sh}_$i.log 2>&1 || { echo "PMC_FAIL $spec $grp"; tail -5 $O/o${ord}_${sh}_$i.log; exit 2; }
  done
done
python3 - "$O" <<'PY'
import csv, glob, os, sys, collections
O = sys.argv[1]
for d in sorted(glob.glob(O + "/o*_*")):
    if not os.path.isdir(d):
        continue
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_imap_tile" in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d), {k: round(sum(v) / len(v), 1) for k, v in sorted(acc.items())})
PY
