// rw_ratio.hip -- HBM rate of streaming kernels by read:write ratio, with no
// conversion at all (not product code).  The widening conversions move R
// written bytes per read byte (1 -> 8: R = 8); this measures what the memory
// system gives such a stream in the product's access shape: a 256-lane block
// reads 16 B per lane (one 4 KiB piece) and writes R x 16 B per lane, every
// wave instruction one contiguous 1 KiB, stores "nt sc1", XCD-contiguous
// blocks; and the mirror for narrowing (R x 16 B read, 16 B written).
// Steady state: 10 launches between events, median of 5 groups, >= 4 GiB.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st16(uint8_t *p, u32x4 w) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}
__device__ __forceinline__ int64_t xcd(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// read 4 KiB, write R x 4 KiB per block
template <int R>
__global__ __launch_bounds__(256) void k_widen(const uint8_t *src, uint8_t *dst, int64_t nblk) {
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= nblk) return;
    u32x4 v = ld16(src + t * 4096 + threadIdx.x * 16);
#pragma unroll
    for (int k = 0; k < R; k++) {
        v.x += k;
        st16(dst + (t * 256 * R + k * 256 + threadIdx.x) * 16, v);
    }
}
// read R x 4 KiB, write 4 KiB per block
template <int R>
__global__ __launch_bounds__(256) void k_narrow(const uint8_t *src, uint8_t *dst, int64_t nblk) {
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= nblk) return;
    u32x4 v[R];
#pragma unroll
    for (int k = 0; k < R; k++) v[k] = ld16(src + (t * 256 * R + k * 256 + threadIdx.x) * 16);
    u32x4 a = v[0];
#pragma unroll
    for (int k = 1; k < R; k++) a ^= v[k];
    st16(dst + t * 4096 + threadIdx.x * 16, a);
}
// write only (the fill kernel's shape), 16 B per lane
__global__ __launch_bounds__(256) void k_write(uint8_t *dst, int64_t nblk) {
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= nblk) return;
    u32x4 v = {(uint32_t)t, 1u, 2u, 3u};
    st16(dst + t * 4096 + threadIdx.x * 16, v);
}
// read only, 16 B per lane
__global__ __launch_bounds__(256) void k_read(const uint8_t *src, int64_t nblk, int *sink) {
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= nblk) return;
    u32x4 v = ld16(src + t * 4096 + threadIdx.x * 16);
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) sink[0] = 1;
}

static float time_it(const std::function<void()> &f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
    f();
    CK(hipDeviceSynchronize());
    for (int g = 0; g < 5; g++) {
        CK(hipEventRecord(a));
        for (int i = 0; i < 10; i++) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float m;
        CK(hipEventElapsedTime(&m, a, b));
        ms.push_back(m / 10);
    }
    std::sort(ms.begin(), ms.end());
    return ms[2];
}

int main(int argc, char **argv) {
    const int64_t moved = (argc > 1 ? atoll(argv[1]) : 4) << 30;
    uint8_t *src, *dst;
    int *sink;
    CK(hipMalloc(&src, moved));
    CK(hipMalloc(&dst, moved));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 0x5a, moved));
    auto rep = [&](const char *name, double bytes, const std::function<void()> &f) {
        const float ms = time_it(f);
        printf("%-16s %8.4f ms %7.1f GB/s %5.1f %%\n", name, ms, bytes / ms / 1e6, bytes / ms / 1e6 / 80.0);
    };
#define WIDEN(R)                                                                                          \
    {                                                                                                     \
        const int64_t nb = moved / (4096 * (1 + R));                                                      \
        rep("read1:write" #R, (double)nb * 4096 * (1 + R),                                                \
            [&] { hipLaunchKernelGGL(k_widen<R>, dim3(nb), dim3(256), 0, 0, src, dst, nb); });            \
    }
#define NARROW(R)                                                                                         \
    {                                                                                                     \
        const int64_t nb = moved / (4096 * (1 + R));                                                      \
        rep("read" #R ":write1", (double)nb * 4096 * (1 + R),                                             \
            [&] { hipLaunchKernelGGL(k_narrow<R>, dim3(nb), dim3(256), 0, 0, src, dst, nb); });           \
    }
    for (int round = 0; round < 2; round++) {
        WIDEN(1) WIDEN(2) WIDEN(4) WIDEN(8) NARROW(2) NARROW(4) NARROW(8)
        {
            const int64_t nb = moved / 4096;
            rep("write only", (double)nb * 4096, [&] { hipLaunchKernelGGL(k_write, dim3(nb), dim3(256), 0, 0, dst, nb); });
            rep("read only", (double)nb * 4096,
                [&] { hipLaunchKernelGGL(k_read, dim3(nb), dim3(256), 0, 0, src, nb, sink); });
        }
    }
    return 0;
}
