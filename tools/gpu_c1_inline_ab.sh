#!/bin/bash
# C1 first touch, host buffers: a 4 MiB put written by the caller with pwrite
# (PNCX_IO_INLINE_MB=16, default) against the pool's mapped tasks (0), with
# and without MAP_POPULATE (PNCX_IO_POPULATE), in-process alternation record
# by record (api_check c1ab), 2 runs each.
#   bash tools/gpu_c1_inline_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
F=/dev/shm/pncx_inline_ab.nc
for pop in 0 1; do
  for run in 1 2; do
    rm -f $F
    echo "populate=$pop $(PNCX_IO_POPULATE=$pop timeout -k 10 120 $R/tests/mpi/api_check c1ab $F 1048576 64 IO_INLINE_MB 16 0)" || exit 1
  done
done
rm -f $F
