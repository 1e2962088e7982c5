# re-entry check after container re-creation: GPU tests, smoke, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -n 40 gpurun_out/t_all.log; exit 3; }
tail -n 2 gpurun_out/t_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -n 30 gpurun_out/smoke.log; exit 4; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -n 30 gpurun_out/bench_default.err; exit 5; }
cat gpurun_out/bench_default.json
