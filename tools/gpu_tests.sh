# GPU step: run the named pytest files (default: all of tests/) with -m gpu,
# one process, per-test time limit; output to gpurun_out/<tag>.txt.
#   tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 1000 python -u -m pytest "${@:-tests}" -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/$tag.txt 2>&1
rc=$?
tail -n 40 gpurun_out/$tag.txt
exit $rc
