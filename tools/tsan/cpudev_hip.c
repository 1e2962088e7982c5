/*
 * The four HIP runtime calls tests/mpi/api_check.c makes itself (device
 * buffers for the *_dev variants), for the ThreadSanitizer build of
 * api_check only (tools/tsan/run_api.sh): the program's "device" buffers are
 * then the CPU stand-in's (tools/tsan/cpudev_stub.c), which the library's
 * pointer queries recognise.  Never linked into the library.
 */
#include <string.h>
#include <hip/hip_runtime_api.h>
#include "../../pnetcdf_amd/csrc/pncx_shim.h"

hipError_t hipMalloc(void **p, size_t n) { return pncxrt_malloc(p, n) == 0 ? hipSuccess : hipErrorOutOfMemory; }
hipError_t hipFree(void *p) { (void)pncxrt_free(p); return hipSuccess; }
hipError_t hipMemcpy(void *d, const void *s, size_t n, hipMemcpyKind k)
{
    (void)k;
    memmove(d, s, n);
    return hipSuccess;
}
hipError_t hipMemset(void *d, int v, size_t n)
{
    memset(d, v, n);
    return hipSuccess;
}
