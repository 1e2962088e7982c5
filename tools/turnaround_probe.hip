// turnaround_probe.hip -- how long does a synchronous "launch, wait, return"
// cost on top of the kernel?  (pncx_dev_batch's whole call vs its kernel.)
// Standalone; not part of the product.  A streaming kernel of a given size
// (out-of-place 4-byte swap, 1024 lanes x 16 B per block) is launched and
// waited for in a loop, with the completion seen through:
//   sync     hipStreamSynchronize
//   evspin   hipEventRecord + hipEventQuery spin (pncx_dev_batch today)
//   flag     a 1-block kernel queued after it stores the call's sequence
//            number into pinned host memory (vector store, system scope);
//            the host spins on that word
//   lastblk  the streaming kernel's last block (per-launch ticket counter)
//            stores the sequence number into pinned host memory itself
// plus the same kernels queued back to back (GPU-side time, no host wait).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 sw(u32x4 v) {
    v.x = __builtin_bswap32(v.x); v.y = __builtin_bswap32(v.y);
    v.z = __builtin_bswap32(v.z); v.w = __builtin_bswap32(v.w);
    return v;
}

template <bool LAST>
__global__ __launch_bounds__(1024) void k_swap(const u32x4 *src, u32x4 *dst, unsigned *ticket,
                                               volatile int *host, int seq) {
    const long long i = (long long)blockIdx.x * 1024 + threadIdx.x;
    __builtin_nontemporal_store(sw(__builtin_nontemporal_load(src + i)), dst + i);
    if constexpr (LAST) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            const unsigned t = atomicAdd(ticket + (blockIdx.x & 7) * 32, 1u);
            // the per-XCD-slot counters; the last of them reports
            const unsigned per = gridDim.x / 8 + ((blockIdx.x & 7) < (gridDim.x & 7) ? 1u : 0u);
            if (t + 1 == per) {
                const unsigned d = atomicAdd(ticket + 8 * 32, 1u);
                if (d + 1 == 8) {
                    for (int k = 0; k <= 8; k++) ticket[k * 32] = 0;
                    __threadfence_system();
                    __hip_atomic_store(host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
}

__global__ void k_flag(volatile int *host, int seq) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double now_us() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main(int argc, char **argv) {
    const int reps = 200;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int *host;
    CK(hipHostMalloc((void **)&host, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *host = 0;
    int *dhost;
    CK(hipHostGetDevicePointer((void **)&dhost, host, 0));
    unsigned *ticket;
    CK(hipMalloc(&ticket, 9 * 32 * 4));
    CK(hipMemset(ticket, 0, 9 * 32 * 4));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const long long sizes[] = {1 << 20, 16 << 20, 768 << 20};   // bytes swapped (read; same written)
    u32x4 *src, *dst;
    CK(hipMalloc(&src, 768 << 20));
    CK(hipMalloc(&dst, 768 << 20));
    CK(hipMemset(src, 0x5a, 768 << 20));
    int seq = 0;
    for (long long bytes : sizes) {
        const unsigned nb = (unsigned)(bytes / (1024 * 16));
        const char *names[] = {"queued", "sync", "evspin", "flag", "lastblk"};
        for (int mode = 0; mode < 5; mode++) {
            std::vector<double> us;
            for (int r = 0; r < reps + 10; r++) {
                const double t0 = now_us();
                seq++;
                if (mode == 4) k_swap<true><<<nb, 1024, 0, st>>>(src, dst, ticket, dhost, seq);
                else k_swap<false><<<nb, 1024, 0, st>>>(src, dst, ticket, dhost, seq);
                if (mode == 0) {
                    if (r == reps + 9) CK(hipStreamSynchronize(st));
                } else if (mode == 1) {
                    CK(hipStreamSynchronize(st));
                } else if (mode == 2) {
                    CK(hipEventRecord(ev, st));
                    while (hipEventQuery(ev) == hipErrorNotReady) {}
                } else {
                    if (mode == 3) k_flag<<<1, 64, 0, st>>>(dhost, seq);
                    while (__atomic_load_n(host, __ATOMIC_ACQUIRE) != seq)
                        if (now_us() - t0 > 1e6) { printf("mode %d: no completion word\n", mode); return 1; }
                }
                const double t1 = now_us();
                if (r >= 10) us.push_back(t1 - t0);
            }
            CK(hipStreamSynchronize(st));
            double tot = 0;
            for (double u : us) tot += u;
            std::sort(us.begin(), us.end());
            printf("%9lld B  %-8s  mean %8.2f us  median %8.2f us  p10 %8.2f  p90 %8.2f\n", bytes, names[mode],
                   tot / us.size(), us[us.size() / 2], us[us.size() / 10], us[us.size() * 9 / 10]);
        }
        // queued: per-launch time = total / reps
        const double t0 = now_us();
        for (int r = 0; r < reps; r++) k_swap<false><<<nb, 1024, 0, st>>>(src, dst, ticket, dhost, 0);
        CK(hipStreamSynchronize(st));
        printf("%9lld B  back-to-back  %8.2f us per launch\n", bytes, (now_us() - t0) / reps);
    }
    CK(hipGetLastError());
    return 0;
}
