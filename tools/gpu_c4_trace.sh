# Kernel trace of the synchronous C4 call (bench.py --workload c4) for
# tools/c4_trace_gaps.py: batch kernel, completion block and the gaps
set -o pipefail
O=${OUT:-gpurun_out/r06e_c4trace}
mkdir -p $O
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $O -o c4 -- python3 bench.py --workload c4 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo TRACE_FAIL; tail -5 $O/bench.err; exit 1; }
f=$(find $O -name "*kernel_trace.csv" | head -1)
python3 tools/c4_trace_gaps.py "$f" | tee $O/gaps.txt
cp "$f" $O/c4_kernel_trace.csv
