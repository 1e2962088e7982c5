// widen_sweep.hip -- tile shapes for the 4:1 / 8:1 conversion classes (not
// product code).  The product stages the narrow side of a 256-lane block
// through LDS with a block barrier (pncx_kern.hpp tile_body, USE_LDS); these
// classes ran at 72-77 % of peak against 82-85 % for 1:1 and 2:1 (round 2).
// Variants, each over >= 4 GiB moved, timed in steady state (10 launches of
// the same kernel between events, median of 5 such groups):
//   blk    the product shape: block tile, LDS, __syncthreads
//   wave   each wave stages its own quarter of the tile in LDS: no block
//          barrier (wave_barrier only orders the wave's own LDS accesses)
//   wave2  as wave, two tiles per wave, both loads issued first
//   direct no LDS: R narrow loads of 16/R bytes per lane (each wave
//          instruction contiguous), R 16-byte stores per lane
//   wave64 as wave with 64-lane blocks (one wave per block)
// Cases: get NC_BYTE -> double (1 -> 8), get NC_SHORT -> double (2 -> 8),
// get NC_BYTE -> float (1 -> 4), put double -> NC_BYTE (8 -> 1, range
// checked, fill -127), put float -> NC_BYTE (4 -> 1).
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

// ---- element ops: narrow (NS bytes) <-> wide (WS bytes) ------------------
struct B2D {   // get NC_BYTE -> double
    static constexpr int NS = 1, WS = 8;
    __device__ static uint64_t w(uint8_t x) { double d = (double)(int8_t)x; uint64_t u; __builtin_memcpy(&u, &d, 8); return u; }
};
struct S2D {   // get NC_SHORT (big-endian) -> double
    static constexpr int NS = 2, WS = 8;
    __device__ static uint64_t w(uint16_t x) { double d = (double)(int16_t)__builtin_bswap16(x); uint64_t u; __builtin_memcpy(&u, &d, 8); return u; }
};
struct B2F {   // get NC_BYTE -> float
    static constexpr int NS = 1, WS = 4;
    __device__ static uint32_t w(uint8_t x) { float f = (float)(int8_t)x; uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
};
struct D2B {   // put double -> NC_BYTE, range checked
    static constexpr int NS = 1, WS = 8;
    __device__ static uint8_t n(uint64_t u, bool &bad) {
        double d; __builtin_memcpy(&d, &u, 8);
        const bool o = d > 127.0 || d < -128.0;
        bad |= o;
        const double ds = d != d ? 0.0 : d;
        return o ? (uint8_t)(int8_t)-127 : (uint8_t)(int8_t)(int32_t)ds;
    }
};
struct F2B {   // put float -> NC_BYTE
    static constexpr int NS = 1, WS = 4;
    __device__ static uint8_t n(uint32_t u, bool &bad) {
        float f; __builtin_memcpy(&f, &u, 4);
        const bool o = f > 127.0f || f < -128.0f;
        bad |= o;
        const float fs = f != f ? 0.0f : f;
        return o ? (uint8_t)(int8_t)-127 : (uint8_t)(int8_t)(int32_t)fs;
    }
};

template <int B> struct UT;
template <> struct UT<1> { typedef uint8_t t; };
template <> struct UT<2> { typedef uint16_t t; };
template <> struct UT<4> { typedef uint32_t t; };
template <> struct UT<8> { typedef uint64_t t; };

// narrow 16/R-byte piece -> wide 16 bytes
template <class Op>
__device__ __forceinline__ u32x4 widen16(const uint8_t *np) {
    constexpr int E = 16 / Op::WS;
    typename UT<Op::NS>::t s[E];
    typename UT<Op::WS>::t d[E];
    __builtin_memcpy(s, np, sizeof s);
#pragma unroll
    for (int e = 0; e < E; e++) d[e] = Op::w(s[e]);
    u32x4 o;
    __builtin_memcpy(&o, d, 16);
    return o;
}
template <class Op>
__device__ __forceinline__ void narrow16(u32x4 v, uint8_t *np, bool &bad) {
    constexpr int E = 16 / Op::WS;
    typename UT<Op::WS>::t s[E];
    typename UT<Op::NS>::t d[E];
    __builtin_memcpy(s, &v, 16);
#pragma unroll
    for (int e = 0; e < E; e++) d[e] = Op::n(s[e], bad);
    __builtin_memcpy(np, d, sizeof d);
}

template <int B> struct NV;
template <> struct NV<2> { typedef uint16_t t; };
template <> struct NV<4> { typedef uint32_t t; };
template <> struct NV<8> { typedef uint64_t t; };

// ---- widening variants: narrow src (n elems), wide dst ---------------------
// blk: 256-lane block = one tile of 256*16 narrow bytes
template <class Op, int L = 256>
__global__ __launch_bounds__(L) void w_blk(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    __shared__ __attribute__((aligned(16))) uint8_t lds[16 * L];
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    const int lane = threadIdx.x;
    *reinterpret_cast<u32x4 *>(lds + lane * 16) = ld16(src + t * 16 * L + lane * 16);
    __syncthreads();
    typename NV<PB>::t w[R];
#pragma unroll
    for (int k = 0; k < R; k++) w[k] = *reinterpret_cast<const typename NV<PB>::t *>(lds + (k * L + lane) * PB);
#pragma unroll
    for (int k = 0; k < R; k++) st16(dst + (t * L * R + k * L + lane) * 16, widen16<Op>((const uint8_t *)&w[k]));
}
// blk with its LDS tile in dynamic shared memory, so the launch can ask for
// more LDS than the tile needs and cap the blocks per CU (occupancy)
template <class Op, int L>
__global__ __launch_bounds__(L) void w_blkd(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    extern __shared__ __attribute__((aligned(16))) uint8_t dlds[];
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    const int lane = threadIdx.x;
    *reinterpret_cast<u32x4 *>(dlds + lane * 16) = ld16(src + t * 16 * L + lane * 16);
    __syncthreads();
    typename NV<PB>::t w[R];
#pragma unroll
    for (int k = 0; k < R; k++) w[k] = *reinterpret_cast<const typename NV<PB>::t *>(dlds + (k * L + lane) * PB);
#pragma unroll
    for (int k = 0; k < R; k++) st16(dst + (t * L * R + k * L + lane) * 16, widen16<Op>((const uint8_t *)&w[k]));
}
template <class Op, int L>
__global__ __launch_bounds__(L) void n_blkd(const uint8_t *src, uint8_t *dst, int64_t ntile, int *flags) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    extern __shared__ __attribute__((aligned(16))) uint8_t dlds[];
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    const int lane = threadIdx.x;
    bool bad = false;
    u32x4 v[R];
#pragma unroll
    for (int k = 0; k < R; k++) v[k] = ld16(src + (t * L * R + k * L + lane) * 16);
#pragma unroll
    for (int k = 0; k < R; k++) {
        uint8_t nb[PB];
        narrow16<Op>(v[k], nb, bad);
        typename NV<PB>::t x;
        __builtin_memcpy(&x, nb, PB);
        *reinterpret_cast<typename NV<PB>::t *>(dlds + (k * L + lane) * PB) = x;
    }
    __syncthreads();
    st16(dst + t * 16 * L + lane * 16, *reinterpret_cast<const u32x4 *>(dlds + lane * 16));
    const unsigned long long m = __ballot(bad);
    if (m && (lane & 63) == (unsigned)(__ffsll((long long)m) - 1)) flags[blockIdx.x] = 1;
}

// 1:1 8-byte swap, 16 B per lane (C2's shape) and NC_INT -> double (C3's
// direct shape: 8 B read, 16 B written per lane), LDS only as occupancy cap
__global__ __launch_bounds__(256) void k_swap8d(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    extern __shared__ uint8_t dlds[];
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    u32x4 v = ld16(src + (t * 256 + threadIdx.x) * 16);
    u32x4 o = {__builtin_bswap32(v.y), __builtin_bswap32(v.x), __builtin_bswap32(v.w), __builtin_bswap32(v.z)};
    if (v.x == 0x12345678u) dlds[threadIdx.x] = 1;
    st16(dst + (t * 256 + threadIdx.x) * 16, o);
}
__global__ __launch_bounds__(256) void k_i2dd(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    extern __shared__ uint8_t dlds[];
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(src + (t * 256 + threadIdx.x) * 8));
    const double a = (double)(int32_t)__builtin_bswap32(v.x), b = (double)(int32_t)__builtin_bswap32(v.y);
    u32x4 o;
    __builtin_memcpy(&o, &a, 8);
    __builtin_memcpy((uint8_t *)&o + 8, &b, 8);
    if (v.x == 0x12345678u) dlds[threadIdx.x] = 1;
    st16(dst + (t * 256 + threadIdx.x) * 16, o);
}

// wave: each wave its own 1 KiB of narrow bytes, no block barrier
template <class Op, int TPW>
__global__ __launch_bounds__(1024) void w_wave(const uint8_t *src, uint8_t *dst, int64_t nwt) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    __shared__ __attribute__((aligned(16))) uint8_t lds[16384 * TPW];
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int64_t wt0 = (xcd(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + wv) * TPW;   // first wave tile
    uint8_t *my = lds + wv * 1024 * TPW;
    u32x4 v[TPW];
#pragma unroll
    for (int u = 0; u < TPW; u++) if (wt0 + u < nwt) v[u] = ld16(src + (wt0 + u) * 1024 + l * 16);
#pragma unroll
    for (int u = 0; u < TPW; u++) *reinterpret_cast<u32x4 *>(my + u * 1024 + l * 16) = v[u];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < TPW; u++) {
        if (wt0 + u >= nwt) break;
        typename NV<PB>::t w[R];
#pragma unroll
        for (int k = 0; k < R; k++) w[k] = *reinterpret_cast<const typename NV<PB>::t *>(my + u * 1024 + (k * 64 + l) * PB);
#pragma unroll
        for (int k = 0; k < R; k++)
            st16(dst + ((wt0 + u) * 64 * R + k * 64 + l) * 16, widen16<Op>((const uint8_t *)&w[k]));
    }
}
// direct: R narrow loads of PB bytes per lane, R stores
template <class Op, int L = 256>
__global__ __launch_bounds__(L) void w_direct(const uint8_t *src, uint8_t *dst, int64_t ntile) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    const int lane = threadIdx.x;
    typename NV<PB>::t w[R];
#pragma unroll
    for (int k = 0; k < R; k++)
        w[k] = __builtin_nontemporal_load(reinterpret_cast<const typename NV<PB>::t *>(src + t * 16 * L + (k * L + lane) * PB));
#pragma unroll
    for (int k = 0; k < R; k++) st16(dst + (t * L * R + k * L + lane) * 16, widen16<Op>((const uint8_t *)&w[k]));
}

// ---- narrowing variants: wide src, narrow dst ------------------------------
template <class Op>
__global__ __launch_bounds__(256) void n_blk(const uint8_t *src, uint8_t *dst, int64_t ntile, int *flags) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    const int lane = threadIdx.x;
    bool bad = false;
    u32x4 v[R];
#pragma unroll
    for (int k = 0; k < R; k++) v[k] = ld16(src + (t * 256 * R + k * 256 + lane) * 16);
#pragma unroll
    for (int k = 0; k < R; k++) {
        uint8_t nb[PB];
        narrow16<Op>(v[k], nb, bad);
        typename NV<PB>::t x;
        __builtin_memcpy(&x, nb, PB);
        *reinterpret_cast<typename NV<PB>::t *>(lds + (k * 256 + lane) * PB) = x;
    }
    __syncthreads();
    st16(dst + t * 4096 + lane * 16, *reinterpret_cast<const u32x4 *>(lds + lane * 16));
    const unsigned long long m = __ballot(bad);
    if (m && (lane & 63) == (unsigned)(__ffsll((long long)m) - 1)) flags[blockIdx.x] = 1;
}
template <class Op, int TPW>
__global__ __launch_bounds__(256) void n_wave(const uint8_t *src, uint8_t *dst, int64_t nwt, int *flags) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096 * TPW];
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int64_t wt0 = (xcd(blockIdx.x, gridDim.x) * (blockDim.x >> 6) + wv) * TPW;
    uint8_t *my = lds + wv * 1024 * TPW;
    bool bad = false;
#pragma unroll
    for (int u = 0; u < TPW; u++) {
        if (wt0 + u >= nwt) break;
        u32x4 v[R];
#pragma unroll
        for (int k = 0; k < R; k++) v[k] = ld16(src + ((wt0 + u) * 64 * R + k * 64 + l) * 16);
#pragma unroll
        for (int k = 0; k < R; k++) {
            uint8_t nb[PB];
            narrow16<Op>(v[k], nb, bad);
            typename NV<PB>::t x;
            __builtin_memcpy(&x, nb, PB);
            *reinterpret_cast<typename NV<PB>::t *>(my + u * 1024 + (k * 64 + l) * PB) = x;
        }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < TPW; u++)
        if (wt0 + u < nwt) st16(dst + (wt0 + u) * 1024 + l * 16, *reinterpret_cast<const u32x4 *>(my + u * 1024 + l * 16));
    const unsigned long long m = __ballot(bad);
    if (m && l == (unsigned)(__ffsll((long long)m) - 1)) flags[blockIdx.x] = 1;
}
template <class Op>
__global__ __launch_bounds__(256) void n_direct(const uint8_t *src, uint8_t *dst, int64_t ntile, int *flags) {
    constexpr int R = Op::WS / Op::NS, PB = 16 / R;
    const int64_t t = xcd(blockIdx.x, gridDim.x);
    if (t >= ntile) return;
    const int lane = threadIdx.x;
    bool bad = false;
    u32x4 v[R];
#pragma unroll
    for (int k = 0; k < R; k++) v[k] = ld16(src + (t * 256 * R + k * 256 + lane) * 16);
#pragma unroll
    for (int k = 0; k < R; k++) {
        uint8_t nb[PB];
        narrow16<Op>(v[k], nb, bad);
        typename NV<PB>::t x;
        __builtin_memcpy(&x, nb, PB);
        __builtin_nontemporal_store(x, reinterpret_cast<typename NV<PB>::t *>(dst + t * 4096 + (k * 256 + lane) * PB));
    }
    const unsigned long long m = __ballot(bad);
    if (m && (lane & 63) == (unsigned)(__ffsll((long long)m) - 1)) flags[blockIdx.x] = 1;
}

// ---- driver -----------------------------------------------------------------
static float time_it(const std::function<void()> &f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
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

static uint8_t *g_src, *g_dst, *g_ref;
static int *g_flags;

template <class Op>
static void widen_case(const char *name, int64_t moved) {
    constexpr int R = Op::WS / Op::NS;
    const int64_t nbytes_n = moved / (1 + R) / 4096 * 4096;      // narrow bytes
    const int64_t ntile = nbytes_n / 4096, nwt = nbytes_n / 1024, wide = nbytes_n * R;
    const double alg = (double)nbytes_n * (1 + R);
    struct V { const char *n; std::function<void()> f; };
    std::vector<V> vs = {
        {"blk", [&] { hipLaunchKernelGGL(w_blk<Op>, dim3(ntile), dim3(256), 0, 0, g_src, g_dst, ntile); }},
        {"wave", [&] { hipLaunchKernelGGL((w_wave<Op, 1>), dim3((nwt + 3) / 4), dim3(256), 0, 0, g_src, g_dst, nwt); }},
        {"wave2", [&] { hipLaunchKernelGGL((w_wave<Op, 2>), dim3((nwt + 7) / 8), dim3(256), 0, 0, g_src, g_dst, nwt); }},
        {"wave64", [&] { hipLaunchKernelGGL((w_wave<Op, 1>), dim3(nwt), dim3(64), 0, 0, g_src, g_dst, nwt); }},
        {"direct", [&] { hipLaunchKernelGGL(w_direct<Op>, dim3(ntile), dim3(256), 0, 0, g_src, g_dst, ntile); }},
        {"blk1024", [&] { hipLaunchKernelGGL((w_blk<Op, 1024>), dim3(ntile / 4), dim3(1024), 0, 0, g_src, g_dst, ntile / 4); }},
        {"wave1024", [&] { hipLaunchKernelGGL((w_wave<Op, 1>), dim3(nwt / 16), dim3(1024), 0, 0, g_src, g_dst, nwt); }},
        {"dir1024", [&] { hipLaunchKernelGGL((w_direct<Op, 1024>), dim3(ntile / 4), dim3(1024), 0, 0, g_src, g_dst, ntile / 4); }},
    };
    for (int rep = 0; rep < 2; rep++)
        for (auto &v : vs) {
            CK(hipMemset(g_dst, 0, wide));
            v.f();
            CK(hipDeviceSynchronize());
            if (v.n[0] == 'b') CK(hipMemcpy(g_ref, g_dst, 1 << 20, hipMemcpyDeviceToDevice));
            else {
                std::vector<uint8_t> a(1 << 20), b(1 << 20);
                CK(hipMemcpy(a.data(), g_ref, 1 << 20, hipMemcpyDeviceToHost));
                CK(hipMemcpy(b.data(), g_dst, 1 << 20, hipMemcpyDeviceToHost));
                if (a != b) printf("  MISMATCH %s %s\n", name, v.n);
            }
            const float ms = time_it(v.f);
            printf("%-22s %-7s %8.4f ms %7.1f GB/s %5.1f %%\n", name, v.n, ms, alg / ms / 1e6, alg / ms / 1e6 / 80.0);
        }
}

template <class Op>
static void narrow_case(const char *name, int64_t moved) {
    constexpr int R = Op::WS / Op::NS;
    const int64_t nbytes_n = moved / (1 + R) / 4096 * 4096;
    const int64_t ntile = nbytes_n / 4096, nwt = nbytes_n / 1024;
    const double alg = (double)nbytes_n * (1 + R);
    struct V { const char *n; std::function<void()> f; };
    std::vector<V> vs = {
        {"blk", [&] { hipLaunchKernelGGL(n_blk<Op>, dim3(ntile), dim3(256), 0, 0, g_src, g_dst, ntile, g_flags); }},
        {"wave", [&] { hipLaunchKernelGGL((n_wave<Op, 1>), dim3((nwt + 3) / 4), dim3(256), 0, 0, g_src, g_dst, nwt, g_flags); }},
        {"wave2", [&] { hipLaunchKernelGGL((n_wave<Op, 2>), dim3((nwt + 7) / 8), dim3(256), 0, 0, g_src, g_dst, nwt, g_flags); }},
        {"wave64", [&] { hipLaunchKernelGGL((n_wave<Op, 1>), dim3(nwt), dim3(64), 0, 0, g_src, g_dst, nwt, g_flags); }},
        {"direct", [&] { hipLaunchKernelGGL(n_direct<Op>, dim3(ntile), dim3(256), 0, 0, g_src, g_dst, ntile, g_flags); }},
    };
    for (int rep = 0; rep < 2; rep++)
        for (auto &v : vs) {
            CK(hipMemset(g_dst, 0, nbytes_n));
            v.f();
            CK(hipDeviceSynchronize());
            if (v.n[0] == 'b') CK(hipMemcpy(g_ref, g_dst, 1 << 20, hipMemcpyDeviceToDevice));
            else {
                std::vector<uint8_t> a(1 << 20), b(1 << 20);
                CK(hipMemcpy(a.data(), g_ref, 1 << 20, hipMemcpyDeviceToHost));
                CK(hipMemcpy(b.data(), g_dst, 1 << 20, hipMemcpyDeviceToHost));
                if (a != b) printf("  MISMATCH %s %s\n", name, v.n);
            }
            const float ms = time_it(v.f);
            printf("%-22s %-7s %8.4f ms %7.1f GB/s %5.1f %%\n", name, v.n, ms, alg / ms / 1e6, alg / ms / 1e6 / 80.0);
        }
}

// occupancy: blocks of L lanes with `lds` bytes of LDS each (>= the tile)
template <class Op, bool widen>
static void occ_case(const char *name, int64_t moved) {
    constexpr int R = Op::WS / Op::NS;
    const int64_t nbytes_n = moved / (1 + R) / 16384 * 16384;
    const double alg = (double)nbytes_n * (1 + R);
    static const int cfg[][2] = {{256, 4096}, {256, 27306}, {256, 32768}, {256, 40960}, {256, 54613},
                                 {256, 81920}, {1024, 16384}, {1024, 98304}};
    for (auto &c : cfg) {
        const int L = c[0], lds = c[1];
        const int64_t ntile = nbytes_n / (16 * L);
        std::function<void()> f;
        if constexpr (widen) {
            if (L == 256) f = [&, lds, ntile] { hipLaunchKernelGGL((w_blkd<Op, 256>), dim3(ntile), dim3(256), lds, 0, g_src, g_dst, ntile); };
            else f = [&, lds, ntile] { hipLaunchKernelGGL((w_blkd<Op, 1024>), dim3(ntile), dim3(1024), lds, 0, g_src, g_dst, ntile); };
        } else {
            if (L == 256) f = [&, lds, ntile] { hipLaunchKernelGGL((n_blkd<Op, 256>), dim3(ntile), dim3(256), lds, 0, g_src, g_dst, ntile, g_flags); };
            else f = [&, lds, ntile] { hipLaunchKernelGGL((n_blkd<Op, 1024>), dim3(ntile), dim3(1024), lds, 0, g_src, g_dst, ntile, g_flags); };
        }
        const int per_cu = std::min(163840 / lds, 2048 / L);
        const float ms = time_it(f);
        printf("%-22s lanes=%4d lds=%6d blocks/CU<=%2d waves/CU<=%2d %8.4f ms %5.1f %%\n", name, L, lds, per_cu,
               per_cu * L / 64, ms, alg / ms / 1e6 / 80.0);
    }
}

static void occ_direct(int64_t moved) {
    static const int ldss[] = {0, 27306, 32768, 40960, 54613, 81920};
    for (int which = 0; which < 2; which++)
        for (int lds : ldss) {
            const int bpl = which == 0 ? 32 : 24;                   // bytes moved per lane
            const int64_t ntile = moved / (256 * (int64_t)bpl);
            std::function<void()> f = which == 0
                ? std::function<void()>([&, lds, ntile] { hipLaunchKernelGGL(k_swap8d, dim3(ntile), dim3(256), lds, 0, g_src, g_dst, ntile); })
                : std::function<void()>([&, lds, ntile] { hipLaunchKernelGGL(k_i2dd, dim3(ntile), dim3(256), lds, 0, g_src, g_dst, ntile); });
            const int per_cu = lds ? std::min(163840 / lds, 8) : 8;
            const float ms = time_it(f);
            const double alg = (double)ntile * 256 * bpl;
            printf("%-22s lanes= 256 lds=%6d blocks/CU<=%2d waves/CU<=%2d %8.4f ms %5.1f %%\n",
                   which == 0 ? "swap8 out-of-place" : "get int->double", lds, per_cu, per_cu * 4, ms, alg / ms / 1e6 / 80.0);
        }
}

__global__ void k_fill(uint64_t *p, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}
// doubles / floats of moderate magnitude so the narrowing cases are mostly in range
__global__ void k_fill_f64(double *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (double)((int)((i * 2654435761u) % 300u) - 150) + 0.25;
}
__global__ void k_fill_f32(float *p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = (float)((int)((i * 2654435761u) % 300u) - 150) + 0.25f;
}

int main(int argc, char **argv) {
    const int64_t moved = (argc > 1 ? atoll(argv[1]) : 4) << 30;
    CK(hipMalloc(&g_src, moved));
    CK(hipMalloc(&g_dst, moved));
    CK(hipMalloc(&g_ref, 1 << 20));
    CK(hipMalloc(&g_flags, 64 << 20));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)g_src, moved / 8, 0x5EEDull);
    CK(hipDeviceSynchronize());
    if (argc > 2 && argv[2][0] == 'o') {
        for (int r = 0; r < 2; r++) occ_direct(moved);
        for (int r = 0; r < 2; r++) {
            occ_case<B2D, true>("get byte->double", moved);
            occ_case<S2D, true>("get short->double", moved);
            occ_case<B2F, true>("get byte->float", moved);
        }
        hipLaunchKernelGGL(k_fill_f64, dim3(4096), dim3(256), 0, 0, (double *)g_src, moved / 8);
        CK(hipDeviceSynchronize());
        for (int r = 0; r < 2; r++) occ_case<D2B, false>("put double->byte", moved);
        hipLaunchKernelGGL(k_fill_f32, dim3(4096), dim3(256), 0, 0, (float *)g_src, moved / 4);
        CK(hipDeviceSynchronize());
        for (int r = 0; r < 2; r++) occ_case<F2B, false>("put float->byte", moved);
        return 0;
    }
    widen_case<B2D>("get byte->double", moved);
    widen_case<S2D>("get short->double", moved);
    widen_case<B2F>("get byte->float", moved);
    hipLaunchKernelGGL(k_fill_f64, dim3(4096), dim3(256), 0, 0, (double *)g_src, moved / 8);
    CK(hipDeviceSynchronize());
    if (argc > 2) return 0;
    narrow_case<D2B>("put double->byte", moved);
    hipLaunchKernelGGL(k_fill_f32, dim3(4096), dim3(256), 0, 0, (float *)g_src, moved / 4);
    CK(hipDeviceSynchronize());
    narrow_case<F2B>("put float->byte", moved);
    return 0;
}
