set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1 || { tail -n 40 gpurun_out/t_all.log; exit 3; }
tail -n 2 gpurun_out/t_all.log
bash tools/gpu_round13.sh
