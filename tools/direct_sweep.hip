// direct_sweep.hip -- the direct (register-only) tile of the 1:1 and 2:1
// conversion classes with more than one tile per lane (not product code).
// The compute-heavy pairs of these classes (float -> (u)int64, NC_BYTE ->
// ushort, the 1-byte range checks) stay at 71-75 % of peak while the
// occupancy sweep (profiles/r03_occupancy_sweep_b.txt) puts the best rate
// near 64-80 KiB in flight per CU; a direct 4 -> 8 tile keeps 1.5 KiB per
// wave, 48 KiB per CU.  Variants: U tiles per lane (loads of all U issued
// first), element semantics from the product (pncx_device.hpp get1/put1).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "../pnetcdf_amd/csrc/pncx_device.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using namespace pncx;

__device__ __forceinline__ void st16(uint8_t *p, uint32_t __attribute__((ext_vector_type(4))) w) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
}
__device__ __forceinline__ int64_t xcd(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}
template <int B> struct VT;
template <> struct VT<16> { typedef uint32_t t __attribute__((ext_vector_type(4))); };
template <> struct VT<8> { typedef uint32_t t __attribute__((ext_vector_type(2))); };
template <> struct VT<4> { typedef uint32_t t; };

// GET xtype -> itype; source element big-endian
template <int XT, int IT>
struct G {
    using SU = typename X<XT>::U;
    using DU = typename I<IT>::U;
    static constexpr int SS = X<XT>::size, DS = I<IT>::size;
    __device__ static DU one(SU s, bool &bad) {
        const typename X<XT>::T xx = bits_to<typename X<XT>::T>(bswap(s));
        return bits_to<DU>(get1<XT, IT>(xx, bad));
    }
};
template <int XT, int IT>
struct P {
    using SU = typename I<IT>::U;
    using DU = typename X<XT>::U;
    static constexpr int SS = I<IT>::size, DS = X<XT>::size;
    __device__ static DU one(SU s, bool &bad) {
        const typename X<XT>::T f = X<XT>::fill();
        return bswap(bits_to<DU>(put1<XT, IT>(bits_to<typename I<IT>::T>(s), f, bad)));
    }
};

// a lane: U tiles, each E = 16/W elements: SB source bytes -> DB dest bytes
template <class Op, int U>
__global__ __launch_bounds__(256) void k_direct(const uint8_t *src, uint8_t *dst, int64_t ntile, int *flags) {
    constexpr int W = Op::SS > Op::DS ? Op::SS : Op::DS, E = 16 / W, SB = E * Op::SS, DB = E * Op::DS;
    const int64_t b = xcd(blockIdx.x, gridDim.x);
    bool bad = false;
    typename VT<SB>::t v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t t = b * U + u;
        if (t < ntile) v[u] = __builtin_nontemporal_load(reinterpret_cast<const typename VT<SB>::t *>(src + (t * 256 + threadIdx.x) * SB));
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t t = b * U + u;
        if (t >= ntile) break;
        typename Op::SU s[E];
        typename Op::DU d[E];
        __builtin_memcpy(s, &v[u], SB);
#pragma unroll
        for (int e = 0; e < E; e++) d[e] = Op::one(s[e], bad);
        typename VT<DB>::t o;
        __builtin_memcpy(&o, d, DB);
        if constexpr (DB == 16) st16(dst + (t * 256 + threadIdx.x) * DB, o);
        else __builtin_nontemporal_store(o, reinterpret_cast<typename VT<DB>::t *>(dst + (t * 256 + threadIdx.x) * DB));
    }
    const unsigned long long m = __ballot(bad);
    if (m && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1)) flags[blockIdx.x] = 1;
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

static uint8_t *g_src, *g_dst;
static int *g_flags;
static int64_t g_moved;

template <class Op, int U>
static void run1(const char *name) {
    constexpr int W = Op::SS > Op::DS ? Op::SS : Op::DS, E = 16 / W;
    const int64_t per_tile = 256LL * E * (Op::SS + Op::DS);
    const int64_t ntile = g_moved / per_tile;
    const int64_t nb = (ntile + U - 1) / U;
    const float ms = time_it([&] { hipLaunchKernelGGL((k_direct<Op, U>), dim3(nb), dim3(256), 0, 0, g_src, g_dst, ntile, g_flags); });
    printf("%-26s U=%d %8.4f ms %5.1f %%\n", name, U, ms, (double)ntile * per_tile / ms / 1e6 / 80.0);
}
template <class Op>
static void run(const char *name) {
    run1<Op, 1>(name);
    run1<Op, 2>(name);
    run1<Op, 4>(name);
}

__global__ void k_fill(uint64_t *p, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main(int argc, char **argv) {
    g_moved = (argc > 1 ? atoll(argv[1]) : 4) << 30;
    CK(hipMalloc(&g_src, g_moved));
    CK(hipMalloc(&g_dst, g_moved));
    CK(hipMalloc(&g_flags, 64 << 20));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)g_src, g_moved / 8, 0x5EEDull);
    CK(hipDeviceSynchronize());
    for (int r = 0; r < 2; r++) {
        run<G<NC_INT, PNCX_ITYPE_DOUBLE>>("get int->double (C3)");
        run<G<NC_FLOAT, PNCX_ITYPE_LONGLONG>>("get float->longlong");
        run<G<NC_FLOAT, PNCX_ITYPE_ULONGLONG>>("get float->ulonglong");
        run<P<NC_INT64, PNCX_ITYPE_FLOAT>>("put int64<-float");
        run<G<NC_BYTE, PNCX_ITYPE_USHORT>>("get byte->ushort");
        run<G<NC_BYTE, PNCX_ITYPE_UCHAR>>("get byte->uchar");
        run<P<NC_BYTE, PNCX_ITYPE_UCHAR>>("put byte<-uchar");
        run<G<NC_BYTE, PNCX_ITYPE_SCHAR>>("get byte->schar (copy)");
    }
    return 0;
}
