// ptr_range_probe.hip -- what the HIP runtime reports for registered and
// pinned host memory: the allocation range attributes and hostPointer, for
// pncxrt_host_dptr_range.  Not product code.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <sys/mman.h>
static void show(const char *what, const void *p) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e1 = hipPointerGetAttribute(&base, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p);
    hipError_t e2 = hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p);
    hipPointerAttribute_t at;
    hipError_t e3 = hipPointerGetAttributes(&at, p);
    void *d = nullptr;
    hipError_t e4 = hipHostGetDevicePointer(&d, (void *)p, 0);
    (void)hipGetLastError();
    printf("%-28s p=%p  range_start=%p (%d) size=%zu (%d)  attrs(%d): type=%d host=%p dev=%p  dptr=%p (%d)\n", what, p,
           base, (int)e1, size, (int)e2, (int)e3, (int)at.type, at.hostPointer, at.devicePointer, d, (int)e4);
}
int main() {
    const size_t pg = 4096;
    char *m = (char *)mmap(NULL, 3 * pg, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    m[0] = m[pg] = m[2 * pg] = 1;
    hipHostRegister(m, pg, hipHostRegisterDefault);
    hipHostRegister(m + 2 * pg, pg, hipHostRegisterDefault);
    show("reg page0 start", m);
    show("reg page0 +100", m + 100);
    show("pageable page1", m + pg);
    show("reg page2 start", m + 2 * pg);
    show("reg page2 last byte", m + 3 * pg - 1);
    char *big = (char *)aligned_alloc(pg, 1 << 22);
    big[0] = 1;
    hipHostRegister(big, 1 << 22, hipHostRegisterDefault);
    show("reg 4MiB +1MiB", big + (1 << 20));
    void *pin = nullptr;
    hipHostMalloc(&pin, 1 << 22, hipHostMallocDefault);
    show("hipHostMalloc +1MiB", (char *)pin + (1 << 20));
    void *dm = nullptr;
    hipMalloc(&dm, 1 << 22);
    show("hipMalloc +1MiB", (char *)dm + (1 << 20));
    return 0;
}
