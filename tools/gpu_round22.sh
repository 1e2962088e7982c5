# 1024-lane swapmix batch kernel: parity, C4 bench, C4 rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ncfile.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mix.txt 2>&1 || { tail -n 60 gpurun_out/t_mix.txt; exit 3; }
tail -n 2 gpurun_out/t_mix.txt
for i in 1 2 3; do
timeout -k 10 200 python bench.py --workload c4 --steps 50 --warmup 5 > gpurun_out/bench_c4_$i.json 2> gpurun_out/bench_c4.err || { tail -n 30 gpurun_out/bench_c4.err; exit 4; }
cat gpurun_out/bench_c4_$i.json
done
timeout -k 10 300 bash tools/gpu_prof_c4.sh > gpurun_out/prof_c4.txt 2>&1 || { tail -n 30 gpurun_out/prof_c4.txt; exit 5; }
cat gpurun_out/prof_c4.txt
