#!/bin/bash
# C1 first-touch medians (api_check c1first, 32 records of 4 MiB) under knob
# settings "NAME=VALUE,NAME=VALUE" (each run twice, interleaved), plus the
# reference sequence's probe line (tools/c1_first_probe P0) for the box.
set -o pipefail
export TMPDIR=/tmp
out=${OUT:-gpurun_out/c1_knobs.txt}
: > "$out"
for pass in 1 2; do
  for cfg in "$@"; do
    env_args=$(echo "$cfg" | tr ',' ' ')
    r=$(env $env_args timeout -k 10 120 tests/mpi/api_check c1first /dev/shm/c1k.nc 1048576 32 0) || exit 1
    echo "$cfg $(echo "$r" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read().splitlines()[-1]); print("put %.3f get %.3f err %d" % (d["put_ms_median"], d["get_ms_median"], d["errors"]))')" >> "$out"
  done
done
rm -f /dev/shm/c1k.nc
