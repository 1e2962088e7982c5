set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4 -o c4 -- python3 $R/bench.py --workload c4 --steps 20 --warmup 3 > $R/gpurun_out/prof4/c4.json 2>&1 || exit 1
grep -E "k_batch|Name|memcpy|Memcpy|fill|Fill" $R/gpurun_out/prof4/c4_kernel_stats.csv | cut -c1-200
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('/root/repo/gpurun_out/prof4/c4_kernel_trace.csv')))
ks=[r for r in rows if 'k_batch' in r['Kernel_Name']]
# gaps between consecutive batch kernels
ks.sort(key=lambda r:int(r['Start_Timestamp']))
prev=None
out=[]
for r in ks[-12:]:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    out.append((r['Kernel_Name'][:40], (e-s)/1e3, (s-prev)/1e3 if prev else 0))
    prev=e
for o in out: print(o)
PY
