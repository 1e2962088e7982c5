# flexible API (derived buftypes): GPU parity, then the full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ls /opt/conda/lib/libmpi.so.12 > gpurun_out/mpi_probe.txt 2>&1
timeout -k 10 600 python tools/flex_bench.py > gpurun_out/flex_bench.txt 2>&1 && timeout -k 10 600 python -u -m pytest tests/test_gpu_flex.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flex.txt 2>&1 || { tail -n 60 gpurun_out/t_flex.txt; exit 3; }
tail -n 3 gpurun_out/t_flex.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.txt 2>&1 || { tail -n 40 gpurun_out/t_all.txt; exit 4; }
tail -n 2 gpurun_out/t_all.txt
