// swap_sweep.hip -- standalone tuning sweep for the 8-byte in-place swap
// (config 2).  Not part of the product; the winner is folded into
// pnetcdf_amd/csrc/pncx_kern.hpp.  Interleaved rounds in one process
// (cdna_hip_programming.md §5.4 rule 24).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <string>
#include <functional>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ u32x4 sw8(u32x4 v) {
    u32x4 r;
    r.x = __builtin_bswap32(v.y); r.y = __builtin_bswap32(v.x);
    r.z = __builtin_bswap32(v.w); r.w = __builtin_bswap32(v.z);
    return r;
}
template <bool NT> __device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NT> __device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}

// A: grid-stride, U vectors per lane per iteration
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_gs(u32x4 *p, int64_t nvec) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = tid;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ld<NT>(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; u++) st<NT>(p + i + u * stride, sw8(v[u]));
    }
    for (; i < nvec; i += stride) st<NT>(p + i, sw8(ld<NT>(p + i)));
}

// B: block-chunked: block b owns [b*chunk, (b+1)*chunk) vectors
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_chunk(u32x4 *p, int64_t nvec, int64_t chunk) {
    const int64_t b0 = (int64_t)blockIdx.x * chunk;
    int64_t e = b0 + chunk;
    if (e > nvec) e = nvec;
    int64_t i = b0 + threadIdx.x;
    for (; i + (U - 1) * 256 < e; i += U * 256) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ld<NT>(p + i + u * 256);
#pragma unroll
        for (int u = 0; u < U; u++) st<NT>(p + i + u * 256, sw8(v[u]));
    }
    for (; i < e; i += 256) st<NT>(p + i, sw8(ld<NT>(p + i)));
}

// C: one-shot (no loop): each lane exactly U vectors, grid = nvec/(256U)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_oneshot(u32x4 *p, int64_t nvec) {
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u * 256 < nvec) v[u] = ld<NT>(p + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u * 256 < nvec) st<NT>(p + base + u * 256, sw8(v[u]));
}

// reference points: out-of-place copy-swap, read-only, write-only
__global__ __launch_bounds__(256) void k_copy(const u32x4 *s, u32x4 *d, int64_t nvec) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = tid;
    for (; i + 3 * stride < nvec; i += 4 * stride) {
        u32x4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], dd = s[i + 3 * stride];
        d[i] = sw8(a); d[i + stride] = sw8(b); d[i + 2 * stride] = sw8(c); d[i + 3 * stride] = sw8(dd);
    }
    for (; i < nvec; i += stride) d[i] = sw8(s[i]);
}
__global__ __launch_bounds__(256) void k_read(const u32x4 *s, int64_t nvec, u32x4 *sink) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    u32x4 acc = {0, 0, 0, 0};
    int64_t i = tid;
    for (; i + 3 * stride < nvec; i += 4 * stride) acc ^= s[i] ^ s[i + stride] ^ s[i + 2 * stride] ^ s[i + 3 * stride];
    for (; i < nvec; i += stride) acc ^= s[i];
    if (acc.x == 0x12345678 && acc.y == 0x9abcdef0) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_write(u32x4 *d, int64_t nvec) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    u32x4 v = {1u, 2u, 3u, (uint32_t)tid};
    for (int64_t i = tid; i < nvec; i += stride) d[i] = v;
}


// D: oneshot with block size BS and XCD-contiguous remap option
template <int U, bool NT, int BS, bool XCDMAP>
__global__ __launch_bounds__(BS) void k_one2(u32x4 *p, int64_t nvec) {
    int64_t b = blockIdx.x;
    if constexpr (XCDMAP) {
        const int64_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8;
        b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    }
    const int64_t base = b * BS * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u * BS < nvec) v[u] = ld<NT>(p + base + u * BS);
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u * BS < nvec) st<NT>(p + base + u * BS, sw8(v[u]));
}
// F: oneshot, U vectors per lane BS apart, loads UNPREDICATED (index clamped
// to the last vector; a predicated load waits on its own), stores predicated;
// XCD-contiguous remap; store cache policy SP: 0 nt builtin, 1 plain,
// 2 "sc1" (drop from L2), 3 "sc0 sc1", 4 "nt sc1" (inline asm vector stores)
template <int SP>
__device__ __forceinline__ void st_pol(u32x4 *p, u32x4 v) {
    if constexpr (SP == 0) __builtin_nontemporal_store(v, p);
    else if constexpr (SP == 1) *p = v;
    else if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (SP == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}
template <int U, int BS, int SP, bool RM = true>
__global__ __launch_bounds__(BS) void k_one3(u32x4 *p, int64_t nvec) {
    int64_t b = blockIdx.x;
    const int64_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = b % 8;
    if (RM) b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    const int64_t base = b * BS * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int64_t i = base + u * BS < nvec ? base + u * BS : nvec - 1;
        v[u] = __builtin_nontemporal_load(p + i);
    }
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u * BS < nvec) st_pol<SP>(p + base + u * BS, sw8(v[u]));
}
// E: oneshot where each lane does U consecutive vectors (32/64B per lane)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_one_consec(u32x4 *p, int64_t nvec) {
    const int64_t base = ((int64_t)blockIdx.x * 256 + threadIdx.x) * U;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u < nvec) v[u] = ld<NT>(p + base + u);
#pragma unroll
    for (int u = 0; u < U; u++) if (base + u < nvec) st<NT>(p + base + u, sw8(v[u]));
}

struct Var {
    std::string name;
    double bytes_factor;  // bytes moved per vector / 16
    std::function<void()> run;
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int64_t nbytes = (int64_t)(gib * (1LL << 30));
    const int64_t nvec = nbytes / 16;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    u32x4 *p, *q, *sink;
    CK(hipMalloc(&p, nbytes));
    CK(hipMalloc(&q, nbytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(p, 0x5a, nbytes));
    CK(hipMemset(q, 0x00, nbytes));
    printf("CUs %d, slab %.2f GiB, rounds %d\n", cus, gib, rounds);

    std::vector<Var> vars;
    auto add = [&](std::string n, double f, std::function<void()> r) { vars.push_back({n, f, r, {}}); };

#define ONE2(U, NT, BS, XM) { const int64_t g = (nvec + (int64_t)BS * U - 1) / ((int64_t)BS * U); \
      add(std::string("one2 U") + #U + " nt" + #NT + " bs" + #BS + " xcd" + #XM, 2, [=] { hipLaunchKernelGGL((k_one2<U, NT, BS, XM>), dim3(g), dim3(BS), 0, 0, p, nvec); }); }
    ONE2(1, true, 256, true)
#define ONE3(U, BS, SP) { const int64_t g = (nvec + (int64_t)BS * U - 1) / ((int64_t)BS * U); \
      add(std::string("one3 U") + #U + " bs" + #BS + " store" + #SP, 2, [=] { hipLaunchKernelGGL((k_one3<U, BS, SP>), dim3(g), dim3(BS), 0, 0, p, nvec); }); }
    ONE3(1, 256, 0) ONE3(1, 256, 4) ONE3(1, 512, 4) ONE3(1, 1024, 4) ONE3(1, 128, 4) ONE3(2, 256, 4)
#define ONE3N(U, BS, SP) { const int64_t g = (nvec + (int64_t)BS * U - 1) / ((int64_t)BS * U); \
      add(std::string("one3 noremap U") + #U + " bs" + #BS + " store" + #SP, 2, [=] { hipLaunchKernelGGL((k_one3<U, BS, SP, false>), dim3(g), dim3(BS), 0, 0, p, nvec); }); }
    ONE3N(1, 256, 4) ONE3N(1, 1024, 4)
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto &v : vars) { v.run(); v.run(); }
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; r++) {
        for (auto &v : vars) {
            CK(hipEventRecord(a, 0));
            v.run();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            v.ms.push_back(ms);
        }
    }
    CK(hipGetLastError());
    for (auto &v : vars) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
        const double bytes = (double)nvec * 16 * v.bytes_factor;
        printf("%-28s median %8.3f ms  %7.1f GB/s   best %7.1f GB/s  (%.1f%% of 8 TB/s)\n", v.name.c_str(), med,
               bytes / med / 1e6, bytes / mn / 1e6, 100.0 * bytes / med / 1e6 / 8000.0);
    }
    return 0;
}
