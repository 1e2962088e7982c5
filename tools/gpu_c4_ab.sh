# GPU tests, then the product batch kernel (tools/c4_placement.py --steady)
# beside the sweep kernels on the same box
set -o pipefail
R=$GRAFT_REPO_ROOT
tag=${1:-c4ab}
bash $R/tools/gpu_tests.sh ${tag}_tests || exit 1
timeout -k 10 200 python -u $R/tools/c4_placement.py --steady > $R/gpurun_out/${tag}_placement.txt 2>&1 || exit 1
timeout -k 10 150 $R/tools/c4_shape_sweep > $R/gpurun_out/${tag}_sweep.txt 2>&1 || exit 1
timeout -k 10 300 python -u $R/bench.py --workload c4 --no-cpu-baseline --steps 20 > $R/gpurun_out/${tag}_bench_c4.json 2>&1 || exit 1
timeout -k 10 300 python -u $R/bench.py --workload c4_erange --no-cpu-baseline --steps 20 > $R/gpurun_out/${tag}_bench_c4e.json 2>&1 || exit 1
cat $R/gpurun_out/${tag}_placement.txt
grep -E "seg  1024 remap true|pool 1024 remap true|flat 1024 remap true" $R/gpurun_out/${tag}_sweep.txt
