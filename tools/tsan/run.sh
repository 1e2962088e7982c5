#!/bin/bash
# Host-side ThreadSanitizer run of the C host code (file layer, I/O pool,
# staging, warm-up) against a synchronous CPU stand-in for the device
# (tools/tsan/cpudev_stub.c, never part of the library), on CPU: tools/tsan/threads.c
# writes and reads one file per thread while another thread churns the
# file table.  Any race report fails the run (exit code 66).
set -eo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/tsan/build
mkdir -p $OUT
CSRC=pnetcdf_amd/csrc
# STUB=nodev: the no-device stub of the ASan build (the no-conversion paths only)
if [ "${STUB:-cpudev}" = nodev ]; then STUB=tools/asan/pncxrt_stub.c; else STUB=tools/tsan/cpudev_stub.c; fi
gcc -O1 -g -fsanitize=thread -fno-omit-frame-pointer -Iinclude -I$CSRC \
    tools/tsan/threads.c $CSRC/pncx_host.c $CSRC/pncx_cdf.c $CSRC/pncx_nc.c $CSRC/pncx_io.c \
    $STUB -o $OUT/threads -lpthread
DIR=$(mktemp -d /dev/shm/pncx_tsan_XXXXXX)
trap 'rm -rf "$DIR"' EXIT
TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1" $OUT/threads "$DIR" ${NTHREADS:-6} ${ITERS:-3}
