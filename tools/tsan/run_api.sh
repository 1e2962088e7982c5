#!/bin/bash
# ThreadSanitizer run of the whole host stack behind the public ncmpi_* API
# (dispatcher, driver, ncmpii layer, file layer, I/O pool) on CPU:
# tests/mpi/api_check's tst_pthread restatement (mode "pthread", one MPI
# process, MPI_THREAD_MULTIPLE) and its 32-thread file-table churn
# ("pthreadhdr"), built with -fsanitize=thread against the synchronous CPU
# stand-in for the device (tools/tsan/cpudev_stub.c, cpudev_hip.c; never
# part of the library).  MPICH itself is not instrumented.  Any race report
# fails the run (exit code 66).
#   tools/tsan/run_api.sh [dev]      dev=1: hipMalloc'ed (stand-in) buffers
set -eo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/tsan/build
mkdir -p $OUT
CSRC=pnetcdf_amd/csrc
MPI_HOME=${MPI_HOME:-/opt/conda}
gcc -O1 -g -fsanitize=thread -fno-omit-frame-pointer -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
    -Iinclude -I$CSRC -I$MPI_HOME/include \
    tests/mpi/api_check.c $CSRC/pnc_dispatch.c $CSRC/pnc_driver.c $CSRC/pncx_mpi.c $CSRC/pncx_ncmpii.c \
    $CSRC/pncx_ncx.c $CSRC/pncx_host.c $CSRC/pncx_cdf.c $CSRC/pncx_nc.c $CSRC/pncx_io.c \
    tools/tsan/cpudev_stub.c tools/tsan/cpudev_hip.c \
    -o $OUT/api_check $MPI_HOME/lib/libmpi.so -Wl,-rpath,$MPI_HOME/lib -lpthread -ldl
DIR=$(mktemp -d /dev/shm/pncx_tsan_api_XXXXXX)
trap 'rm -rf "$DIR"' EXIT
export TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1"
DEV=${1:-0}
# the reference's 4 x 5 and 1 MiB records (staged pipelines), collective and independent
$OUT/api_check pthread "$DIR/a" 6 4 5 1 $DEV
$OUT/api_check pthread "$DIR/b" 6 262144 4 0 $DEV
$OUT/api_check pthreadhdr "$DIR/h" 16 40
echo "api tsan ok dev=$DEV"
