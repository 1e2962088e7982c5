# C4: the product batch kernel and the sweep kernels timed the same ways on one box
#   per-launch events, back-to-back events, and rocprof kernel-trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c4m
mkdir -p $O
timeout -k 10 200 python -u $R/tools/c4_placement.py --steady > $O/placement_steady.txt 2>&1 || exit 1
timeout -k 10 150 $R/tools/c4_shape_sweep > $O/sweep.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sweep -o sweep -- $R/tools/c4_shape_sweep > $O/sweep_under_rocprof.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_place -o place -- python3 $R/tools/c4_placement.py --steady --rounds 3 > $O/placement_under_rocprof.txt 2>&1 || exit 1
cat $O/placement_steady.txt $O/sweep.txt
