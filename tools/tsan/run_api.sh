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
# SAN=address builds with AddressSanitizer + UBSan instead (same programs;
# leak checking off: MPICH's own allocations at exit are not the library's).
set -eo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/tsan/build
mkdir -p $OUT
CSRC=pnetcdf_amd/csrc
MPI_HOME=${MPI_HOME:-/opt/conda}
SAN=${SAN:-thread}
if [ "$SAN" = address ]; then FLAGS="-fsanitize=address,undefined -fno-sanitize-recover=undefined"; BIN=api_check_asan
else FLAGS=-fsanitize=thread; BIN=api_check; fi
gcc -O1 -g $FLAGS -fno-omit-frame-pointer -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
    -Iinclude -I$CSRC -I$MPI_HOME/include \
    tests/mpi/api_check.c $CSRC/pnc_dispatch.c $CSRC/pnc_driver.c $CSRC/pncx_mpi.c $CSRC/pncx_ncmpii.c \
    $CSRC/pncx_ncx.c $CSRC/pncx_host.c $CSRC/pncx_cdf.c $CSRC/pncx_nc.c $CSRC/pncx_io.c \
    tools/tsan/cpudev_stub.c tools/tsan/cpudev_hip.c \
    -o $OUT/$BIN $MPI_HOME/lib/libmpi.so -Wl,-rpath,$MPI_HOME/lib -lpthread -ldl
DIR=$(mktemp -d /dev/shm/pncx_tsan_api_XXXXXX)
trap 'rm -rf "$DIR"' EXIT
export TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1"
export ASAN_OPTIONS="detect_leaks=0 abort_on_error=1" UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1"
DEV=${1:-0}
# the reference's 4 x 5 and 1 MiB records (staged pipelines), collective and independent
$OUT/$BIN pthread "$DIR/a" 6 4 5 1 $DEV
$OUT/$BIN pthread "$DIR/b" 6 262144 4 0 $DEV
$OUT/$BIN pthreadhdr "$DIR/h" 16 40
# single-threaded programs over the same-type paths the stand-in carries out
# (BASELINE configs 1, 4 and 5 at small sizes, the put_vara benchmark,
# define mode, the dispatcher's error returns)
head -c $((128 * 4096 * 2)) /dev/urandom > "$DIR/s.bin"
head -c $((128 * 4096 * 4)) /dev/urandom > "$DIR/f.bin"
$OUT/$BIN c4 "$DIR/c4.nc" "$DIR/s.bin" "$DIR/f.bin" 4096 0 $DEV > /dev/null
$OUT/$BIN c1first "$DIR/c1.nc" 262144 8 $DEV > /dev/null
$OUT/$BIN c1bench "$DIR/c1b.nc" 262144 3 $DEV > /dev/null
$OUT/$BIN records "$DIR/rec.nc" 8 4096 > /dev/null
$OUT/$BIN putvara "$DIR/pv.nc" 4 64 3 1 > /dev/null
$OUT/$BIN putvara "$DIR/pv2.nc" 4 64 3 0 > /dev/null
$OUT/$BIN header "$DIR/hd.nc" > /dev/null
$OUT/$BIN errors "$DIR" > /dev/null
echo "api $SAN ok dev=$DEV"
