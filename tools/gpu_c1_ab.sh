#!/bin/bash
# In-process A/B of libpncx knobs on the C1 first-touch pattern
# (api_check c1ab): arguments "KNOB:A:B[:ENV=V,...]", each run twice.
set -o pipefail
export TMPDIR=/tmp
out=${OUT:-gpurun_out/c1_ab.txt}
: > "$out"
for pass in 1 2; do
  for spec in "$@"; do
    IFS=: read -r knob a b envs <<< "$spec"
    env_args=$(echo "$envs" | tr ',' ' ')
    echo "$spec $(env $env_args timeout -k 10 120 tests/mpi/api_check c1ab /dev/shm/c1ab.nc 1048576 64 $knob $a $b | tail -1)" >> "$out" || exit 1
  done
done
rm -f /dev/shm/c1ab.nc
