# reference programs restated: put_all_kinds, iput_all_kinds, test_fillvalue, tst_def_var_fill, scalar
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_reftests_nonblocking.py tests/test_gpu_all_kinds.py tests/test_gpu_reftests_file.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t31.txt 2>&1 || { tail -n 80 gpurun_out/t31.txt; exit 3; }
tail -n 30 gpurun_out/t31.txt
