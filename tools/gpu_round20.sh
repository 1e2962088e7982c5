# ncmpidiff (first-difference kernel) + flex/imap parity
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ncmpidiff.py tests/test_gpu_flex.py tests/test_gpu_imap.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_diff.txt 2>&1 || { tail -n 60 gpurun_out/t_diff.txt; exit 3; }
tail -n 3 gpurun_out/t_diff.txt
