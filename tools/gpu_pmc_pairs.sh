# rocprofv3 counters for the slowest conversion pairs (VERDICT r2 "do this" 2):
# a timing pass, then separate PMC passes (SQ instruction/cycle counters,
# FETCH_SIZE, WRITE_SIZE), each under its own time limit.
#   bash tools/gpu_pmc_pairs.sh <tag> <pairs>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1
PAIRS=$2
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
M="python3 $R/tools/matrix_bench.py --pairs $PAIRS --reps 5"
timeout -k 10 180 $M > $O/time.jsonl 2> $O/time.err || { echo TIME_FAIL; tail -5 $O/time.err; exit 1; }
cat $O/time.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O/sq -o sq -- $M > $O/sq.log 2>&1 || { echo SQ_FAIL; tail -5 $O/sq.log; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/sq2 -o sq2 -- $M > $O/sq2.log 2>&1 || { echo SQ2_FAIL; tail -5 $O/sq2.log; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o fetch -- $M > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $O/fetch.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o write -- $M > $O/write.log 2>&1 || { echo WRITE_FAIL; tail -5 $O/write.log; exit 5; }
find $O -name "*.csv" | sort
