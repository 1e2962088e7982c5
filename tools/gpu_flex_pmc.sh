# HBM traffic of the pack kernels: FETCH_SIZE and WRITE_SIZE passes over
# tools/flex_bench.py --big (--reps 1), summarised per kernel into
# gpurun_out/<tag>_flex_pmc/summary.txt by tools/flex_pmc_summary.py.
#   bash tools/gpu_flex_pmc.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1_flex_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o fetch -- python3 $R/tools/flex_bench.py --big --reps 1 > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o write -- python3 $R/tools/flex_bench.py --big --reps 1 > $O/write.log 2>&1 || { echo WRITE_FAIL; tail -5 $O/write.log; exit 2; }
python3 $R/tools/flex_pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
find $O -name "*.csv" -size +2M -delete
