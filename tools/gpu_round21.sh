# full GPU suite + smoke + default bench after the ncmpidiff kernel landed; diff kernel rate
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.txt 2>&1 || { tail -n 60 gpurun_out/t_all.txt; exit 3; }
tail -n 2 gpurun_out/t_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -n 30 gpurun_out/smoke.log; exit 4; }
tail -n 2 gpurun_out/smoke.log
timeout -k 10 300 python tools/diff_bench.py > gpurun_out/diff_bench.txt 2>&1 || { tail -n 30 gpurun_out/diff_bench.txt; exit 5; }
cat gpurun_out/diff_bench.txt
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -n 30 gpurun_out/bench_default.err; exit 6; }
cat gpurun_out/bench_default.json
