set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/prof_c4 -o c4 -- python bench.py --workload c4 --steps 20 --warmup 3 > gpurun_out/bench_c4_prof.json 2> gpurun_out/bench_c4_prof.err || { tail -n 30 gpurun_out/bench_c4_prof.err; exit 1; }
cat gpurun_out/bench_c4_prof.json
find gpurun_out/prof_c4 -name "*stats*.csv" | head
