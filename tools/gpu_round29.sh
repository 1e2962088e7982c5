# k_imap / k_tmap_runs streaming stores: flex parity + bench; then the rocprof/PMC evidence refresh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flex.py tests/test_gpu_imap.py tests/test_gpu_reftests_file.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flex.txt 2>&1 || { tail -n 60 gpurun_out/t_flex.txt; exit 3; }
tail -n 1 gpurun_out/t_flex.txt
timeout -k 10 300 python tools/flex_bench.py > gpurun_out/flex_bench.txt 2>&1 || exit 4
grep -h GB_per_s gpurun_out/flex_bench.txt | cut -c1-120
rm -rf gpurun_out/prof
bash tools/gpu_profile.sh > gpurun_out/profile.txt 2>&1 || { tail -n 40 gpurun_out/profile.txt; exit 5; }
grep '"metric"' gpurun_out/profile.txt | cut -c1-200
