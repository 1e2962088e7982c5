// c2_lane_sweep.hip -- block size and block order for the in-place 8-byte
// swap (config 2).  Standalone; not part of the product (k_tile: 256 lanes,
// XCD-contiguous order, one 16 B vector per lane, nt loads, "nt sc1" stores).
// On the C4 sweep 1024-lane blocks in XCD-contiguous order ran 0.4-0.8
// points ahead of 256-lane ones (tools/c4_shape_sweep.hip); this checks the
// headline shape.  Variants: L lanes in {256, 512, 1024} x order:
//   seq    launch order
//   xcd    XCD-contiguous (each XCD one contiguous run of tiles, k_tile's)
//   chunk  XCD-interleaved chunks of 64 tiles (all XCDs near each other)
//   xcd/S  each XCD walks S sub-ranges of its range side by side (8 S streams)
//   xcdxG  G XCDs share one range, tiles interleaved (8 / G streams)
// Result (profiles/r02s_c2_order_sweep.txt): 8 streams (xcd, xcdx2, chunk at
// 1024 lanes) 85.0-85.4 %; 16 / 32 streams 79.6-80.4 / 75.0-75.6 %.
// over S GiB in place (argv[1], default 32), splitmix64 data, 10 launches
// back to back per sample, interleaved rounds.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 sw8(u32x4 v) {
    u32x4 r;
    r.x = __builtin_bswap32(v.y); r.y = __builtin_bswap32(v.x);
    r.z = __builtin_bswap32(v.w); r.w = __builtin_bswap32(v.z);
    return r;
}

__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

template <int ORD>
__device__ __forceinline__ long long order(long long b, long long nb) {
    if constexpr (ORD == 0) return b;
    if constexpr (ORD == 1) {
        const long long q = nb >> 3, r = nb & 7, x = b & 7;
        return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
    }
    if constexpr (ORD == 2) {
        // chunks of 64 tiles dealt round-robin over the 8 XCDs: block b (XCD b & 7)
        // takes tile (b >> 3) % 64 of chunk ((b >> 3) / 64) * 8 + (b & 7); the
        // grid is a multiple of 512 blocks here
        const long long x = b & 7, k = b >> 3;
        return ((k >> 6) * 8 + x) * 64 + (k & 63);
    }
    if constexpr (ORD == 3 || ORD == 4) {
        // XCD-contiguous, but each XCD's range split into S = 2 / 4 sub-ranges
        // walked side by side (8 S concurrent streams instead of 8); the grid
        // is a multiple of 8 S blocks here
        constexpr long long S = ORD == 3 ? 2 : 4;
        const long long x = b & 7, k = b >> 3, per = nb >> 3;
        return x * per + (k % S) * (per / S) + k / S;
    }
    // ORD = 5 / 6: G = 2 / 4 XCDs share one contiguous range (8 / G streams),
    // their blocks interleaved tile by tile
    constexpr long long G = ORD == 5 ? 2 : 4;
    const long long x = b & 7, k = b >> 3, per = nb / (8 / G);
    return (x / G) * per + k * G + (x % G);
}

template <int L, int ORD>
__global__ __launch_bounds__(L) void k_sw(u32x4 *p) {
    const long long i = order<ORD>(blockIdx.x, gridDim.x) * L + threadIdx.x;
    st(p + i, sw8(__builtin_nontemporal_load(p + i)));
}

__global__ void k_rand(uint64_t *p, long long n, uint64_t seed) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct V { std::string n; int lanes; void (*f)(u32x4 *, long long); std::vector<float> ms; };

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 32.0;
    const long long bytes = (long long)(gib * (1ll << 30)) / (1 << 20) * (1 << 20);
    u32x4 *p;
    CK(hipMalloc(&p, bytes));
    k_rand<<<8192, 256>>>((uint64_t *)p, bytes / 8, 2);
    std::vector<V> vs;
#define VAR(L, O, NM) vs.push_back({std::string(NM) + " " #L, L, [](u32x4 *q, long long nb) { k_sw<L, O><<<nb, L>>>(q); }, {}});
    VAR(256, 1, "xcd") VAR(512, 1, "xcd") VAR(1024, 1, "xcd")
    VAR(256, 0, "seq") VAR(1024, 0, "seq")
    VAR(256, 2, "chunk") VAR(1024, 2, "chunk")
    VAR(256, 3, "xcd/2") VAR(1024, 3, "xcd/2")
    VAR(256, 5, "xcdx2") VAR(256, 6, "xcdx4") VAR(1024, 5, "xcdx2") VAR(1024, 6, "xcdx4")
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 4;
    for (int r = 0; r < 6; r++)
        for (auto &v : vs) {
            const long long nb = bytes / (v.lanes * 16);
            v.f(p, nb);
            CK(hipEventRecord(e0));
            for (int k = 0; k < reps; k++) v.f(p, nb);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) v.ms.push_back(ms / reps);
        }
    CK(hipGetLastError());
    printf("in-place 8-byte swap, %.1f GiB\n", bytes / (double)(1ll << 30));
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
        printf("%-12s median %.4f ms  %.1f GB/s  (%.1f%%)  best %.1f%%\n", v.n.c_str(), med, 2.0 * bytes / med / 1e6,
               2.0 * bytes / med / 1e6 / 80.0, 2.0 * bytes / best / 1e6 / 80.0);
    }
    return 0;
}
