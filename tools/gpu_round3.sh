set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof3
timeout -k 10 400 python tools/matrix_bench.py --all > gpurun_out/matrix_all.log 2>&1 || exit 21
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof3/c4.json 2>&1 || exit 22
grep -E "k_batch|Name" $GRAFT_REPO_ROOT/gpurun_out/prof3/c4_kernel_stats.csv | cut -c1-250
