// Does the CPU see what a kernel stored into pinned host memory once an
// event recorded after the kernel has completed?  (Round 6: after host-buffer
// puts the file held 64-byte pieces of a staging region's previous content;
// the staging region is hipHostMalloc'ed memory the conversion kernel writes
// over PCIe, and the host pwrites it after hipEventSynchronize.)
//
// ROUNDS times per variant: the CPU fills the buffer with a stale pattern,
// a kernel stores this round's pattern into it (plain or nontemporal
// stores), the host waits (event sync / stream sync / event query spin) and
// checks every 64-byte line.
//   hipcc --offload-arch=gfx950 -O2 tools/visibility_probe.hip -o tools/visibility_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <bool NT>
__global__ void k_fill(unsigned *dst, size_t n, unsigned v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (NT) __builtin_nontemporal_store(v ^ (unsigned)i, dst + i);
        else dst[i] = v ^ (unsigned)i;
    }
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? atol(argv[1]) : (1 << 20);
    const int rounds = argc > 2 ? atoi(argv[2]) : 300;
    const char *kinds[] = {"hostmalloc-default", "hostmalloc-coherent", "hostmalloc-noncoherent", "register"};
    const unsigned hflags[] = {hipHostMallocDefault, hipHostMallocCoherent, hipHostMallocNonCoherent, 0};
    const char *waits[] = {"event_sync", "stream_sync", "event_query_spin"};
    hipStream_t s;
    hipEvent_t ev;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    for (int k = 0; k < 4; k++)
        for (int nt = 0; nt < 2; nt++)
            for (int w = 0; w < 3; w++) {
                unsigned *h, *hd;
                if (k < 3) CK(hipHostMalloc((void **)&h, n * 4, hflags[k]));
                else {
                    h = (unsigned *)aligned_alloc(4096, n * 4);
                    CK(hipHostRegister(h, n * 4, hipHostRegisterMapped));
                }
                CK(hipHostGetDevicePointer((void **)&hd, h, 0));
                long long bad_rounds = 0, bad_lines = 0;
                for (int r = 1; r <= rounds; r++) {
                    const unsigned v = (unsigned)r * 2654435761u;
                    memset(h, 0xEE, n * 4);                         // the stale content
                    if (nt) k_fill<true><<<1024, 256, 0, s>>>(hd, n, v);
                    else k_fill<false><<<1024, 256, 0, s>>>(hd, n, v);
                    CK(hipEventRecord(ev, s));
                    if (w == 0) CK(hipEventSynchronize(ev));
                    else if (w == 1) CK(hipStreamSynchronize(s));
                    else while (hipEventQuery(ev) == hipErrorNotReady) {}
                    long long lines = 0;
                    for (size_t i = 0; i < n; i += 16) {
                        int ok = 1;
                        for (size_t j = i; j < i + 16 && j < n; j++)
                            if (h[j] != (v ^ (unsigned)j)) { ok = 0; break; }
                        lines += !ok;
                    }
                    if (lines) { bad_rounds++; bad_lines += lines; }
                }
                printf("{\"kind\": \"%s\", \"stores\": \"%s\", \"wait\": \"%s\", \"rounds\": %d, \"bad_rounds\": %lld, "
                       "\"bad_lines\": %lld}\n", kinds[k], nt ? "nontemporal" : "plain", waits[w], rounds, bad_rounds,
                       bad_lines);
                fflush(stdout);
                if (k < 3) CK(hipHostFree(h));
                else { CK(hipHostUnregister(h)); free(h); }
            }
    return 0;
}
