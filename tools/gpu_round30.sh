# byte stores plain again: full GPU suite, then the 220-pair matrix with nt sc1 stores
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.txt 2>&1 || { tail -n 60 gpurun_out/t_all.txt; exit 3; }
tail -n 1 gpurun_out/t_all.txt
timeout -k 10 600 python tools/matrix_bench.py --all > gpurun_out/matrix_all.log 2>&1 || { tail -n 20 gpurun_out/matrix_all.log; exit 4; }
tail -n 3 gpurun_out/matrix_all.log
