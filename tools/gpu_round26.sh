# async batch: parity + C4 bench sync vs async + rocprof of the async run
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_par.txt 2>&1 || { tail -n 60 gpurun_out/t_par.txt; exit 3; }
tail -n 2 gpurun_out/t_par.txt
timeout -k 10 200 python bench.py --workload c4 --steps 50 --warmup 5 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -n 30 gpurun_out/bench_c4.err; exit 4; }
timeout -k 10 200 python bench.py --workload c4 --async-batch --steps 50 --warmup 5 > gpurun_out/bench_c4_async.json 2> gpurun_out/bench_c4.err || { tail -n 30 gpurun_out/bench_c4.err; exit 5; }
cat gpurun_out/bench_c4.json gpurun_out/bench_c4_async.json
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_c4a
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4a -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --async-batch --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_c4a.json 2>&1 || exit 6
grep k_batch $GRAFT_REPO_ROOT/gpurun_out/prof_c4a/c4_kernel_stats.csv
