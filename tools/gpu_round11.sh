set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
df -h /dev/shm > gpurun_out/shm.txt 2>&1 || true
timeout -k 10 600 python tools/file_bench.py --big-gib 1 > gpurun_out/file_bench.json 2> gpurun_out/file_bench.err || { tail -n 30 gpurun_out/file_bench.err; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail -n 30 gpurun_out/bench_c2.err; exit 2; }
cat gpurun_out/shm.txt gpurun_out/file_bench.json gpurun_out/bench_c2.json
