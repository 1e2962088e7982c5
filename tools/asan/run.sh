#!/bin/bash
# Host-side AddressSanitizer run of the C host code (header codec, file
# layer, I/O pool, dispatch) with a no-device stub shim, on CPU.
set -eo pipefail
cd "$(dirname "$0")/../.."
OUT=tools/asan/build
mkdir -p $OUT
CSRC=pnetcdf_amd/csrc
gcc -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fPIC -shared -Iinclude -I$CSRC \
    $CSRC/pncx_host.c $CSRC/pncx_cdf.c $CSRC/pncx_nc.c $CSRC/pncx_io.c tools/asan/pncxrt_stub.c \
    -o $OUT/libpncx.so -lpthread
export PNCX_LIB_PATH=$PWD/$OUT/libpncx.so
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=1
export LSAN_OPTIONS=suppressions=$PWD/tools/asan/lsan.supp:print_suppressions=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
PNCX_NO_TORCH=1 LD_PRELOAD=$(gcc -print-file-name=libasan.so) python3 tools/asan/workload.py
