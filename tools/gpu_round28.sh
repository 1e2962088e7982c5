# nt sc1 streaming stores: full parity, then every bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.txt 2>&1 || { tail -n 60 gpurun_out/t_all.txt; exit 3; }
tail -n 1 gpurun_out/t_all.txt
for w in c2 c3 c4; do
timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench.err || { tail -n 20 gpurun_out/bench.err; exit 4; }
done
timeout -k 10 300 python bench.py --workload c4 --async-batch --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c4_async.json 2> gpurun_out/bench.err || exit 5
for w in c2 c3 c4 c4_async; do python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_avg'])"; done
timeout -k 10 300 python tools/fill_bench.py > gpurun_out/fill_bench.txt 2>&1 || exit 6
timeout -k 10 300 python tools/flex_bench.py > gpurun_out/flex_bench.txt 2>&1 || exit 7
timeout -k 10 300 python tools/align_bench.py > gpurun_out/align_after.txt 2>&1 || exit 8
grep -h GBps gpurun_out/fill_bench.txt gpurun_out/align_after.txt | cut -c1-150
grep -h GB_per_s gpurun_out/flex_bench.txt | cut -c1-120
