# rocprofv3 kernel-trace stats of the default bench.py run (all workloads);
#   tools/gpu_prof_bench.sh <tag> [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof_$tag
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
f=$(find $O -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(r["Name"][:110], r["Calls"], r["AverageNs"], sep=" | ")
PY
