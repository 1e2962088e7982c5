// conv_sweep.hip -- tuning sweep for the fused 4-byte swap + int32->double
// (config 3): store-pattern variants.  Not product code.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <string>
#include <functional>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <class T, bool NT> __device__ __forceinline__ T ld(const T *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
// built twice: plain nt stores, and with -DSC1 "nt sc1" stores (write-through, line not kept in L2)
template <class T, bool NT> __device__ __forceinline__ void st(T *p, T v) {
#ifdef SC1
    if constexpr (NT && sizeof(T) == 16) {
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
        return;
    } else if constexpr (NT && sizeof(T) == 8) {
        asm volatile("global_store_dwordx2 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
        return;
    }
#endif
    if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}
__device__ __forceinline__ double cv(uint32_t be) { return (double)(int32_t)__builtin_bswap32(be); }
__device__ __forceinline__ int64_t xcd(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// A: 16B load (4 ints) -> 2 x 16B stores at lane*32 (interleaved)
template <bool NT, bool XM>
__global__ __launch_bounds__(256) void kA(const u32x4 *s, f64x2 *d, int64_t nv) {
    const int64_t b = XM ? xcd(blockIdx.x, gridDim.x) : blockIdx.x;
    const int64_t v = b * 256 + threadIdx.x;
    if (v >= nv) return;
    u32x4 x = ld<u32x4, NT>(s + v);
    f64x2 o0 = {cv(x.x), cv(x.y)}, o1 = {cv(x.z), cv(x.w)};
    st<f64x2, NT>(d + 2 * v, o0);
    st<f64x2, NT>(d + 2 * v + 1, o1);
}
// B: 8B load (2 ints) -> 16B store, both contiguous per instruction; U steps
template <bool NT, int U>
__global__ __launch_bounds__(256) void kB(const u32x2 *s, f64x2 *d, int64_t n2) {
    const int64_t b = xcd(blockIdx.x, gridDim.x);
    const int64_t base = b * 256 * U + threadIdx.x;
    u32x2 x[U];
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u * 256 < n2) x[u] = ld<u32x2, NT>(s + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u * 256 < n2) { f64x2 o = {cv(x[u].x), cv(x[u].y)}; st<f64x2, NT>(d + base + u * 256, o); }
}
// C: 16B load, cross-lane permute so each store instruction is contiguous
template <bool NT>
__global__ __launch_bounds__(256) void kC(const u32x4 *s, f64x2 *d, int64_t nv) {
    const int64_t b = xcd(blockIdx.x, gridDim.x);
    const int64_t wave0 = b * 256 + (threadIdx.x & ~63);      // first vector of this wave
    const int lane = threadIdx.x & 63;
    const int64_t v = wave0 + lane;
    u32x4 x = {0, 0, 0, 0};
    if (v < nv) x = ld<u32x4, NT>(s + v);
    // output pair p (16B) of this wave = ints 2p, 2p+1 of the wave's 256 ints
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int p = j * 64 + lane;                // pair index within the wave
        const int src = p >> 1;                     // lane holding ints 2p..2p+1
        const int hi = p & 1;                       // which half of its 4 ints
        uint32_t a0 = __shfl(x.x, src), a1 = __shfl(x.y, src), a2 = __shfl(x.z, src), a3 = __shfl(x.w, src);
        const uint32_t e0 = hi ? a2 : a0, e1 = hi ? a3 : a1;
        const int64_t op = (wave0 * 2) + p;         // output pair index
        if (op < 2 * nv) { f64x2 o = {cv(e0), cv(e1)}; st<f64x2, NT>(d + op, o); }
    }
}
// D: LDS staged: block loads 4 KB (16B/lane), each lane stores 2 contiguous 16B pairs
template <bool NT>
__global__ __launch_bounds__(256) void kD(const u32x4 *s, f64x2 *d, int64_t nv) {
    __shared__ u32x4 lds[256];
    const int64_t b = xcd(blockIdx.x, gridDim.x);
    const int64_t v = b * 256 + threadIdx.x;
    if (v < nv) lds[threadIdx.x] = ld<u32x4, NT>(s + v);
    __syncthreads();
    const uint32_t *li = (const uint32_t *)lds;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int p = j * 256 + threadIdx.x;        // pair within block (512 pairs)
        const int64_t op = b * 512 + p;
        if (op < 2 * nv) { f64x2 o = {cv(li[2 * p]), cv(li[2 * p + 1])}; st<f64x2, NT>(d + op, o); }
    }
}
// G: LDS-DMA staged: each wave global_load_lds 16 B/lane (1 KiB of ints) into
// its own LDS slice, waits for it, then 2 x (8-byte LDS read -> 16-byte store)
// per lane, each store instruction contiguous
template <bool NT>
__global__ __launch_bounds__(256) void kG(const u32x4 *s, f64x2 *d, int64_t nv) {
    __shared__ u32x4 lds[256];
    const int64_t b = xcd(blockIdx.x, gridDim.x);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t v0 = b * 256 + w * 64;                   // first vector of this wave
    if (v0 + 63 < nv) {
        __builtin_amdgcn_global_load_lds((const void *)(s + v0 + lane), (void __attribute__((address_space(3))) *)(lds + w * 64), 16, 0, NT ? 2 : 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t *li = (const uint32_t *)(lds + w * 64);
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int p = k * 64 + lane;                   // pair within the wave (128 pairs)
            f64x2 o = {cv(li[2 * p]), cv(li[2 * p + 1])};
            st<f64x2, NT>(d + 2 * v0 + p, o);
        }
    }
}
// E: 4B load -> 8B store
template <bool NT>
__global__ __launch_bounds__(256) void kE(const uint32_t *s, double *d, int64_t n) {
    const int64_t b = xcd(blockIdx.x, gridDim.x);
    const int64_t i = b * 256 + threadIdx.x;
    if (i < n) st<double, NT>(d + i, cv(ld<uint32_t, NT>(s + i)));
}

struct Var { std::string name; std::function<void()> run; std::vector<float> ms; };

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : (1LL << 31);   // ints
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    uint32_t *s; double *d;
    CK(hipMalloc(&s, n * 4));
    CK(hipMalloc(&d, n * 8));
    CK(hipMemset(s, 0x3c, n * 4));
    std::vector<Var> vars;
    auto add = [&](std::string nm, std::function<void()> r) { vars.push_back({nm, r, {}}); };
    const int64_t nv = n / 4, n2 = n / 2;
    const int64_t gA = (nv + 255) / 256;
    add("A 16B ld, 2x16B interleaved st nt xcd", [=] { hipLaunchKernelGGL((kA<true, true>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("A nt0 xcd", [=] { hipLaunchKernelGGL((kA<false, true>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("A nt1 noxcd", [=] { hipLaunchKernelGGL((kA<true, false>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("B 8B ld 16B st U1 nt", [=] { hipLaunchKernelGGL((kB<true, 1>), dim3((n2 + 255) / 256), dim3(256), 0, 0, (const u32x2 *)s, (f64x2 *)d, n2); });
    add("B U2 nt", [=] { hipLaunchKernelGGL((kB<true, 2>), dim3((n2 + 511) / 512), dim3(256), 0, 0, (const u32x2 *)s, (f64x2 *)d, n2); });
    add("B U4 nt", [=] { hipLaunchKernelGGL((kB<true, 4>), dim3((n2 + 1023) / 1024), dim3(256), 0, 0, (const u32x2 *)s, (f64x2 *)d, n2); });
    add("B U2 nt0", [=] { hipLaunchKernelGGL((kB<false, 2>), dim3((n2 + 511) / 512), dim3(256), 0, 0, (const u32x2 *)s, (f64x2 *)d, n2); });
    add("C shfl contiguous nt", [=] { hipLaunchKernelGGL((kC<true>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("D LDS staged nt", [=] { hipLaunchKernelGGL((kD<true>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("D LDS staged nt0", [=] { hipLaunchKernelGGL((kD<false>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("G LDS-DMA staged nt", [=] { hipLaunchKernelGGL((kG<true>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("G LDS-DMA staged nt0", [=] { hipLaunchKernelGGL((kG<false>), dim3(gA), dim3(256), 0, 0, (const u32x4 *)s, (f64x2 *)d, nv); });
    add("E 4B->8B nt", [=] { hipLaunchKernelGGL((kE<true>), dim3((n + 255) / 256), dim3(256), 0, 0, (const uint32_t *)s, d, n); });
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (auto &v : vars) { v.run(); v.run(); }
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; r++)
        for (auto &v : vars) {
            CK(hipEventRecord(a, 0)); v.run(); CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); v.ms.push_back(ms);
        }
    CK(hipGetLastError());
    for (auto &v : vars) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2];
        const double bytes = 12.0 * n;
        printf("%-40s median %8.3f ms  %7.1f GB/s (%.1f%%)\n", v.name.c_str(), med, bytes / med / 1e6, bytes / med / 1e6 / 80.0);
    }
    return 0;
}
