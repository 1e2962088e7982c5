# checkpoint: full GPU suite, smoke, default bench, N=2 gloo rehearsal of the multi-rank path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.txt 2>&1 || { tail -n 60 gpurun_out/t_all.txt; exit 3; }
tail -n 2 gpurun_out/t_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -n 30 gpurun_out/smoke.log; exit 4; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -n 30 gpurun_out/bench_default.err; exit 6; }
cat gpurun_out/bench_default.json
PNCX_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --slab-gib 2 --gather-gib 0.25 --no-cpu-baseline > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { tail -n 30 gpurun_out/bench_n2_gloo.err; exit 7; }
cat gpurun_out/bench_n2_gloo.json
