# Short-run typemaps (flex_bench --big --short-only): k_tgap (PNCX_TGAP
# default) against k_imap (PNCX_TGAP=0) in alternating runs, then the HBM
# bytes of each workload from one FETCH_SIZE and one WRITE_SIZE pass.
#   bash tools/gpu_short_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1_short
mkdir -p $O
for i in 1 2; do
  for g in -1 0; do
    PNCX_TGAP=$g timeout -k 10 240 python3 $R/tools/flex_bench.py --big --short-only --reps 5 > $O/ab_g$g.$i.json 2> $O/ab_g$g.$i.err || { echo FAIL $g; tail -5 $O/ab_g$g.$i.err; exit 1; }
    echo "TGAP=$g run $i"; cat $O/ab_g$g.$i.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o fetch -- python3 $R/tools/flex_bench.py --big --short-only --reps 1 > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $O/fetch.log; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o write -- python3 $R/tools/flex_bench.py --big --short-only --reps 1 > $O/write.log 2>&1 || { echo WRITE_FAIL; tail -5 $O/write.log; exit 3; }
python3 $R/tools/flex_pmc_seq.py $O 1 > $O/summary.txt && cat $O/summary.txt
find $O -name "*.csv" -size +2M -delete
