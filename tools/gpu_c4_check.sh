set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r02s_tests3 || exit 1
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/prof3
mkdir -p $O
for w in c4 c4_erange c4_async; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o $w -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 3 > $O/$w.json 2> $O/$w.err || { tail -5 $O/$w.err; exit 1; }
  tail -1 $O/$w.json
done
