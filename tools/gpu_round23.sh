# short-run typemaps: per-element offset map (tmode 4) vs table search; parity then perf
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flex.py tests/test_gpu_imap.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flex.txt 2>&1 || { tail -n 60 gpurun_out/t_flex.txt; exit 3; }
tail -n 2 gpurun_out/t_flex.txt
timeout -k 10 300 python tools/flex_bench.py > gpurun_out/flex_bench.txt 2>&1 || { tail -n 30 gpurun_out/flex_bench.txt; exit 4; }
cat gpurun_out/flex_bench.txt
