set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/matrix_bench.py --all --n 268435456 > gpurun_out/matrix.log 2>&1 || exit 21
timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 3 > gpurun_out/bench_c3.json 2>&1 || exit 22
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 > gpurun_out/bench_c4.json 2>&1 || exit 23
cat gpurun_out/matrix.log gpurun_out/bench_c3.json gpurun_out/bench_c4.json
