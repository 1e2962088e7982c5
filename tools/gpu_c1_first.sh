#!/bin/bash
# C1 first-touch legs with per-phase times (api_check c1first, PNCX_PHASES=1),
# under knob settings given as arguments "NAME=VALUE,NAME=VALUE ..." (one run each).
set -o pipefail
export TMPDIR=/tmp
out=${OUT:-gpurun_out/c1first_phases.txt}
: > "$out"
for cfg in "$@"; do
  for th in 8 1; do
    env_args=$(echo "$cfg" | tr ',' ' ')
    echo "# cfg=$cfg threads=$th" >> "$out"
    env $env_args PNCX_PHASES=1 PNCX_IO_THREADS=$th timeout -k 10 120 tests/mpi/api_check c1first /dev/shm/c1f.nc 1048576 32 0 >> "$out" 2>&1 || exit 1
  done
done
rm -f /dev/shm/c1f.nc
