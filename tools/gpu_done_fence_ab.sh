# C4 synchronous completion: the swap-only flag stored relaxed by one wave
# (PNCX_DONE_FENCE=0) against the completion block's system-scope release (1):
# in-process A/B through bench.py's call (tools/c4_done_ab.py) and the C-level
# harness in whole processes (tools/c4_call_c), alternating
# (historical: the knob it A/Bs was removed after the run; kept as the record of how its profiles/ file was made)
set -o pipefail
O=${OUT:-gpurun_out/r06l_done_fence_ab.txt}
mkdir -p gpurun_out
: > $O
timeout -k 10 300 python3 tools/c4_done_ab.py --knob DONE_FENCE --rounds 6 --steps 100 >> $O 2>&1 || exit 1
for r in 1 2 3; do
  for f in 1 0 0 1; do
    echo "fence $f" >> $O
    PNCX_DONE_FENCE=$f timeout -k 10 120 tools/c4_call_c 200 20 >> $O 2>&1 || exit 2
  done
done
PNCX_DONE_FENCE=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "batch" -p no:cacheprovider >> $O 2>&1 || exit 3
