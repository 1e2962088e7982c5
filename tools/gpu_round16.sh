set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1 || { tail -n 40 gpurun_out/t_all.log; exit 3; }
tail -n 2 gpurun_out/t_all.log
for w in c4 c2 c3; do timeout -k 10 600 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -n 30 gpurun_out/bench_$w.err; exit 4; }; done
cat gpurun_out/bench_c4.json gpurun_out/bench_c2.json gpurun_out/bench_c3.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4b -o c4b --output-format csv -- python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4_prof.json 2> gpurun_out/bench_c4_prof.err || { tail -n 30 gpurun_out/bench_c4_prof.err; exit 5; }
find gpurun_out/prof_c4b -name "*stats*" | head
