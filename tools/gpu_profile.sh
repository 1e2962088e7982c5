# rocprofv3 evidence for bench.py: kernel-trace stats and separate FETCH_SIZE /
# WRITE_SIZE PMC passes for the C2 (headline), C3, C4 and C4 ERANGE workloads
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof
mkdir -p $O
for w in c2 c3 c4 c4_erange; do
  A="--workload $w --no-cpu-baseline"
  # the batch workloads as bench.py times them by default: 20 untimed + 200 timed calls
  case $w in c4*) S="--steps 200 --warmup 20";; *) S="--steps 10 --warmup 2";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o $w -- python3 $R/bench.py $A $S > $O/trace_$w.json 2> $O/trace_$w.err || { echo TRACE_FAIL $w; tail -5 $O/trace_$w.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_$w -o $w -- python3 $R/bench.py $A --steps 3 --warmup 1 > $O/pmc_fetch_$w.json 2> $O/pmc_fetch_$w.err || { echo PMC1_FAIL $w; tail -5 $O/pmc_fetch_$w.err; exit 2; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write_$w -o $w -- python3 $R/bench.py $A --steps 3 --warmup 1 > $O/pmc_write_$w.json 2> $O/pmc_write_$w.err || { echo PMC2_FAIL $w; tail -5 $O/pmc_write_$w.err; exit 3; }
  cat $O/trace_$w.json
done
find $O -name "*.csv" | sort
