# C4 synchronous completion: kernel-stamped event (PNCX_DONE_EVENT=1) against
# the completion block (0); then the batch parity tests with the event on
# (historical: the knob it A/Bs was removed after the run; kept as the record of how its profiles/ file was made)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/c4_done_ab.py --rounds 6 --steps 100 > gpurun_out/r06h_done_ab.txt 2>&1 || exit 1
PNCX_DONE_EVENT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "batch" -p no:cacheprovider >> gpurun_out/r06h_done_ab.txt 2>&1 || exit 2
