# reverted imap kernels: parity; then the full rocprof evidence (trace + PMC) for c2/c3/c4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flex.py tests/test_gpu_imap.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flex.txt 2>&1 || { tail -n 60 gpurun_out/t_flex.txt; exit 3; }
tail -n 2 gpurun_out/t_flex.txt
bash tools/gpu_profile.sh > gpurun_out/profile.txt 2>&1 || { tail -n 40 gpurun_out/profile.txt; exit 4; }
cat gpurun_out/profile.txt
