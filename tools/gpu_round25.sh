# batch kernel timing hook: parity + C4 bench (kernel vs call time) + rocprof C4 trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_par.txt 2>&1 || { tail -n 60 gpurun_out/t_par.txt; exit 3; }
tail -n 2 gpurun_out/t_par.txt
timeout -k 10 200 python bench.py --workload c4 --steps 50 --warmup 5 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -n 30 gpurun_out/bench_c4.err; exit 4; }
cat gpurun_out/bench_c4.json
cd /tmp && export TMPDIR=/tmp
rm -rf $GRAFT_REPO_ROOT/gpurun_out/prof_c4b
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4b -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_c4b.json 2>&1 || exit 5
cat $GRAFT_REPO_ROOT/gpurun_out/prof_c4b.json
grep k_batch $GRAFT_REPO_ROOT/gpurun_out/prof_c4b/c4_kernel_stats.csv
