// Does a kernel see what the CPU wrote into pinned host memory since the
// previous kernel read it?  (Round 6: the file-layer fuzz saw stale values
// in a nonblocking get whose external bytes sit in the file layer's pinned
// arena, filled by pread between launches.)
//
// For each allocation kind (hipHostMalloc default / coherent / non-coherent,
// hipHostRegister'ed malloc): ROUNDS times, the CPU fills the buffer with
// the round number, a kernel copies it to device memory reading it over
// PCIe, and the host waits either with hipStreamSynchronize or the library's
// way (a second kernel stores a host-mapped flag the host polls).  Then the
// device copy is checked: every word must hold this round's value.
//   hipcc --offload-arch=gfx950 -O2 tools/coherence_probe.hip -o /tmp/coherence_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_copy(const unsigned *src, unsigned *dst, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
__global__ void k_flag(int *flag, int v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_check(const unsigned *d, size_t n, unsigned want, unsigned *bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (d[i] != want) atomicAdd(bad, 1u);
}

int main(int argc, char **argv) {
    const size_t n = (argc > 1 ? atol(argv[1]) : 1 << 20);       // words (4 MiB)
    const int rounds = argc > 2 ? atoi(argv[2]) : 200;
    const char *kinds[] = {"hostmalloc-default", "hostmalloc-coherent", "hostmalloc-noncoherent", "register"};
    const unsigned flags[] = {hipHostMallocDefault, hipHostMallocCoherent, hipHostMallocNonCoherent, 0};
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *d, *dbad, hbad;
    int *hflag, *dflag;
    CK(hipMalloc(&d, n * 4));
    CK(hipMalloc(&dbad, 4));
    CK(hipHostMalloc((void **)&hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void **)&dflag, hflag, 0));
    for (int k = 0; k < 4; k++) {
        for (int wait = 0; wait < 2; wait++) {
            unsigned *h, *hd;
            if (k < 3) CK(hipHostMalloc((void **)&h, n * 4, flags[k]));
            else {
                h = (unsigned *)aligned_alloc(4096, n * 4);
                CK(hipHostRegister(h, n * 4, hipHostRegisterMapped));
            }
            CK(hipHostGetDevicePointer((void **)&hd, h, 0));
            long long stale_rounds = 0, stale_words = 0;
            for (int r = 1; r <= rounds; r++) {
                const unsigned v = (unsigned)(r * 2654435761u) | 1u;
                for (size_t i = 0; i < n; i++) h[i] = v;               // the CPU writes (pread's role)
                k_copy<<<1024, 256, 0, s>>>(hd, d, n);                  // zero-copy read over PCIe
                if (wait == 0) {
                    CK(hipStreamSynchronize(s));
                } else {                                               // the library's completion word
                    *(volatile int *)hflag = 0;
                    k_flag<<<1, 64, 0, s>>>(dflag, r);
                    while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != r) {}
                }
                CK(hipMemsetAsync(dbad, 0, 4, s));
                k_check<<<1024, 256, 0, s>>>(d, n, v, dbad);
                CK(hipMemcpyAsync(&hbad, dbad, 4, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                if (hbad) { stale_rounds++; stale_words += hbad; }
            }
            printf("{\"kind\": \"%s\", \"wait\": \"%s\", \"rounds\": %d, \"words\": %zu, \"stale_rounds\": %lld, "
                   "\"stale_words\": %lld}\n", kinds[k], wait ? "flag" : "stream_sync", rounds, n, stale_rounds,
                   stale_words);
            fflush(stdout);
            if (k < 3) CK(hipHostFree(h));
            else { CK(hipHostUnregister(h)); free(h); }
        }
    }
    return 0;
}
