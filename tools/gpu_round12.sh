set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1 || { tail -n 40 gpurun_out/t_all.log; exit 3; }
tail -n 2 gpurun_out/t_all.log
for t in 4 8 16; do PNCX_IO_THREADS=$t timeout -k 10 600 python tools/file_bench.py --big-gib 1 > gpurun_out/file_bench_t$t.json 2> gpurun_out/file_bench.err || { tail -n 30 gpurun_out/file_bench.err; exit 1; }; done
cat gpurun_out/file_bench_t*.json
