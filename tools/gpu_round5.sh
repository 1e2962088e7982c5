set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 ./tools/swap_sweep 32 9 > gpurun_out/sweep3.log 2>&1 || exit 31
cat gpurun_out/sweep3.log
PNCX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --slab-gib 4 > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { tail -20 gpurun_out/bench_n2_gloo.err; exit 32; }
grep metric gpurun_out/bench_n2_gloo.json
