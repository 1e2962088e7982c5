// rw_shape.hip -- access shapes for a 1:R read:write (widening) or R:1
// (narrowing) stream with no conversion (not product code).  rw_ratio.hip
// found the product's shape (256-lane block reads one 4 KiB piece and
// writes R x 4 KiB, XCD-contiguous blocks) at 67 % of peak for 1:8 and 71 %
// for 1:4 while write-only runs at 88 % and read-only at 91 %.  Variants:
//   remap   XCD-contiguous block order (1) or launch order (0)
//   wmaj    store order: k-major over the block (0: chunk k*L + lane) or
//           wave-major (1: each wave writes its own contiguous R KiB)
//   tpb     tiles per block, loads of all tiles issued first
//   lanes   block size
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
__device__ __forceinline__ void st16nt(uint8_t *p, u32x4 w) {
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
}
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}
__device__ __forceinline__ int64_t xcd(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// widening: a tile = L lanes x 16 B read, R x L x 16 B written
template <int R, bool REMAP, bool WMAJ, int TPB, int L, bool SC1>
__global__ __launch_bounds__(L) void k_w(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    const int64_t b = REMAP ? xcd(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int lane = threadIdx.x, wv = lane >> 6, l = lane & 63;
    u32x4 v[TPB];
#pragma unroll
    for (int u = 0; u < TPB; u++) {
        const int64_t t = b * TPB + u;
        if (t < ntile) v[u] = ld16(src + (t * L + lane) * 16);
    }
#pragma unroll
    for (int u = 0; u < TPB; u++) {
        const int64_t t = b * TPB + u;
        if (t >= ntile) break;
#pragma unroll
        for (int k = 0; k < R; k++) {
            v[u].x += 1;
            const int64_t c = WMAJ ? (int64_t)wv * 64 * R + k * 64 + l : (int64_t)k * L + lane;
            if (SC1) st16(dst + (t * L * R + c) * 16, v[u]);
            else st16nt(dst + (t * L * R + c) * 16, v[u]);
        }
    }
}
// narrowing: R x L x 16 B read, L x 16 B written
template <int R, bool REMAP, bool WMAJ, int TPB, int L>
__global__ __launch_bounds__(L) void k_n(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    const int64_t b = REMAP ? xcd(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int lane = threadIdx.x, wv = lane >> 6, l = lane & 63;
    u32x4 a[TPB];
#pragma unroll
    for (int u = 0; u < TPB; u++) {
        const int64_t t = b * TPB + u;
        u32x4 v[R];
#pragma unroll
        for (int k = 0; k < R; k++) {
            const int64_t c = WMAJ ? (int64_t)wv * 64 * R + k * 64 + l : (int64_t)k * L + lane;
            v[k] = t < ntile ? ld16(src + (t * L * R + c) * 16) : u32x4{0, 0, 0, 0};
        }
        a[u] = v[0];
#pragma unroll
        for (int k = 1; k < R; k++) a[u] ^= v[k];
    }
#pragma unroll
    for (int u = 0; u < TPB; u++) {
        const int64_t t = b * TPB + u;
        if (t < ntile) st16(dst + (t * L + lane) * 16, a[u]);
    }
}

// the product's direct 2:1 widening shape: 8 B read and 16 B written per lane
template <int L, bool REMAP>
__global__ __launch_bounds__(L) void k_w2d(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const int64_t t = REMAP ? xcd(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    if (t >= ntile) return;
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(src + (t * L + threadIdx.x) * 8));
    u32x4 w = {v.x, v.y, v.x + 1, v.y + 1};
    st16(dst + (t * L + threadIdx.x) * 16, w);
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

static uint8_t *src, *dst;
static int64_t moved;

template <int R, bool REMAP, bool WMAJ, int TPB, int L, bool SC1 = true>
static void W(const char *tag) {
    const int64_t ntile = moved / ((int64_t)L * 16 * (1 + R));
    const int64_t nb = (ntile + TPB - 1) / TPB;
    const double bytes = (double)ntile * L * 16 * (1 + R);
    const float ms = time_it([&] { hipLaunchKernelGGL((k_w<R, REMAP, WMAJ, TPB, L, SC1>), dim3(nb), dim3(L), 0, 0, src, dst, ntile); });
    printf("read1:write%d remap=%d wmaj=%d tpb=%d lanes=%4d %s %-10s %8.4f ms %5.1f %%\n", R, REMAP, WMAJ, TPB, L,
           SC1 ? "ntsc1" : "nt   ", tag, ms, bytes / ms / 1e6 / 80.0);
}
template <int R, bool REMAP, bool WMAJ, int TPB, int L>
static void N(const char *tag) {
    const int64_t ntile = moved / ((int64_t)L * 16 * (1 + R));
    const int64_t nb = (ntile + TPB - 1) / TPB;
    const double bytes = (double)ntile * L * 16 * (1 + R);
    const float ms = time_it([&] { hipLaunchKernelGGL((k_n<R, REMAP, WMAJ, TPB, L>), dim3(nb), dim3(L), 0, 0, src, dst, ntile); });
    printf("read%d:write1 remap=%d wmaj=%d tpb=%d lanes=%4d %-10s %8.4f ms %5.1f %%\n", R, REMAP, WMAJ, TPB, L, tag, ms,
           bytes / ms / 1e6 / 80.0);
}

template <int L, bool REMAP>
static void W2D(const char *tag) {
    const int64_t ntile = moved / ((int64_t)L * 24);
    const double bytes = (double)ntile * L * 24;
    const float ms = time_it([&] { hipLaunchKernelGGL((k_w2d<L, REMAP>), dim3(ntile), dim3(L), 0, 0, src, dst, ntile); });
    printf("read8B:write16B direct remap=%d lanes=%4d %-10s %8.4f ms %5.1f %%\n", REMAP, L, tag, ms, bytes / ms / 1e6 / 80.0);
}

int main(int argc, char **argv) {
    moved = (argc > 1 ? atoll(argv[1]) : 4) << 30;
    CK(hipMalloc(&src, moved));
    CK(hipMalloc(&dst, moved));
    CK(hipMemset(src, 0x5a, moved));
    const bool only2 = argc > 2 && argv[2][0] == '2';
    for (int round = 0; round < 2 && only2; round++) {
        W2D<256, true>("product");
        W2D<512, true>("");
        W2D<1024, true>("");
        W<2, true, false, 1, 256>("");
        W<2, true, false, 1, 1024>("");
        W<1, true, false, 1, 256>("");
        W<1, true, false, 1, 1024>("");
        N<2, true, false, 1, 256>("");
        N<2, true, false, 1, 1024>("");
    }
    for (int round = 0; round < 2 && !only2; round++) {
        W<8, true, false, 1, 256>("product");
        W<8, false, false, 1, 256>("");
        W<8, true, true, 1, 256>("");
        W<8, true, false, 2, 256>("");
        W<8, true, false, 4, 256>("");
        W<8, true, false, 1, 64>("");
        W<8, true, false, 1, 512>("");
        W<8, true, false, 1, 1024>("");
        W<8, false, false, 1, 1024>("");
        W<8, true, false, 1, 256, false>("");
        W<8, false, false, 1, 256, false>("");
        W<4, true, false, 1, 256>("product");
        W<4, false, false, 1, 256>("");
        W<4, true, true, 1, 256>("");
        W<4, true, false, 2, 256>("");
        W<4, true, false, 1, 1024>("");
        W<4, true, false, 1, 256, false>("");
        N<8, true, false, 1, 256>("product");
        N<8, false, false, 1, 256>("");
        N<8, true, true, 1, 256>("");
        N<8, true, false, 2, 256>("");
        N<8, true, false, 1, 1024>("");
        N<4, true, false, 1, 256>("product");
        N<4, false, false, 1, 256>("");
        N<4, true, true, 1, 256>("");
    }
    return 0;
}
