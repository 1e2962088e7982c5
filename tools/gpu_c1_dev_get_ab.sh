#!/bin/bash
# C1 first touch, device buffers: the small get's read in pieces copied up as
# they land (default) against one read then one copy (PNCX_READ_SPLIT=0),
# in-process alternation record by record (api_check c1ab), 3 runs.
#   bash tools/gpu_c1_dev_get_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
F=/dev/shm/pncx_devget_ab.nc
for run in 1 2 3; do
  rm -f $F
  timeout -k 10 120 $R/tests/mpi/api_check c1ab $F 1048576 64 READ_SPLIT 4 0 1 || exit 1
  timeout -k 10 120 $R/tests/mpi/api_check c1ab $F 1048576 64 READ_SPLIT 4 0 0 || exit 1
done
rm -f $F
