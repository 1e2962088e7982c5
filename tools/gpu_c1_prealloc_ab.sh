#!/bin/bash
# C1 first touch with the append preallocation on and off (PNCX_PREALLOC),
# whole processes alternating (an in-process alternation would hand the
# preallocated pages of an "on" record to the next "off" record).
#   bash tools/gpu_c1_prealloc_ab.sh [rounds]
# (the preallocation and its knob were removed after this A/B, commit 676ec1c;
# the script reproduces profiles/r05q_prealloc_ab.txt on 62480bf)
set -o pipefail
R=$GRAFT_REPO_ROOT
F=/dev/shm/pncx_pre_ab.nc
for round in $(seq 1 ${1:-3}); do
  for dev in 0 1; do
    for pre in 1 0 0 1; do
      rm -f $F
      out=$(PNCX_PREALLOC=$pre timeout -k 10 60 $R/tests/mpi/api_check c1first $F 1048576 32 $dev) || { echo "FAIL dev $dev pre $pre"; exit 1; }
      python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'round': $round, 'dev': $dev, 'prealloc': $pre, 'put_ms': d['put_ms_median'], 'get_ms': d['get_ms_median'], 'put_loop_ms': d['put_loop_ms'], 'errors': d['errors']}))" "$out"
    done
  done
done
rm -f $F
