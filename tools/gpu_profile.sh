# rocprofv3 evidence for bench.py (kernel-trace stats + separate PMC passes)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c2 -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/trace_c2.json 2> $O/trace_c2.err || { echo TRACE_FAIL; tail -5 $O/trace_c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o c2 -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { echo PMC1_FAIL; tail -5 $O/pmc_fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o c2 -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write.json 2> $O/pmc_write.err || { echo PMC2_FAIL; tail -5 $O/pmc_write.err; exit 1; }
timeout -k 10 300 python3 $R/bench.py --workload c3 --steps 10 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err || exit 12
timeout -k 10 300 python3 $R/bench.py --workload c4 --steps 10 --warmup 3 > $O/bench_c4.json 2> $O/bench_c4.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c3c4 -- python3 $R/bench.py --workload c3 --steps 3 --warmup 1 > $O/trace_c3.json 2>&1 || exit 14
cat $O/trace_c2.json $O/bench_c3.json $O/bench_c4.json
find $O -name "*.csv" | head -30
