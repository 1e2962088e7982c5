set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ncfile.py -m gpu -q -x > gpurun_out/t_nc.log 2>&1 || { tail -n 60 gpurun_out/t_nc.log; exit 1; }
tail -n 3 gpurun_out/t_nc.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1 || { tail -n 40 gpurun_out/t_all.log; exit 3; }
tail -n 2 gpurun_out/t_all.log
