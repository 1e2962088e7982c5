set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -n 30 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
PNCX_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 3 --warmup 1 --slab-gib 2 --gather-gib 0.25 --no-cpu-baseline > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { tail -n 30 gpurun_out/bench_n2_gloo.err; exit 2; }
cat gpurun_out/bench_n2_gloo.json
for kb in 256 1024 65536; do PNCX_PIN_MIN_KB=$kb timeout -k 10 600 python tools/file_bench.py --big-gib 1 > gpurun_out/file_bench_pin$kb.json 2> gpurun_out/file_bench.err || { tail -n 30 gpurun_out/file_bench.err; exit 3; }; done
for kb in 256 1024 65536; do echo pin$kb; python -c "import json;d=json.load(open('gpurun_out/file_bench_pin$kb.json'));print({k:(v.get('put_s'),v.get('get_s'),v.get('ours_s')) for k,v in d.items() if isinstance(v,dict)})"; done
