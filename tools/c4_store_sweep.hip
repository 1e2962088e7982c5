// c4_store_sweep.hip -- load/store cache policy for the C4-sized swap batch.
// Standalone; not part of the product.  768 MiB out-of-place 4-byte swap
// (1.5 GiB moved, the C4 batch's bytes) as one flat buffer pair and as 256
// buffers (2/4 MiB alternating, one hipMalloc each, block -> buffer by the
// group rule of k_batch_swapmix), 1024 lanes x 16 B per block, with
//   loads:  nt (nontemporal builtin) | plain
//   stores: nt | nt sc1 (inline asm) | plain
// plus persistent blocks that prefetch their next tile (all 65-74 %:
// profiles/r02_c4_store_sweep.txt).  Launches queued back to back (20 per
// sample); interleaved rounds.  Sources hold splitmix64 bits: with memset
// patterns (round 1's sweeps) plain stores looked best, with random bits
// they lose (the product's bench inputs are random).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Seg { const u32x4 *src; u32x4 *dst; long long block0; int es; int pad; };

__device__ __forceinline__ u32x4 sw(u32x4 v, int es) {
    u32x4 r;
    if (es == 2) {
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = ((v[k] & 0x00ff00ffu) << 8) | ((v[k] >> 8) & 0x00ff00ffu);
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = __builtin_bswap32(v[k]);
    }
    return r;
}

template <int LD>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (LD == 0) return __builtin_nontemporal_load(p);
    else return *p;
}
template <int ST>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if constexpr (ST == 0) __builtin_nontemporal_store(v, p);
    else if constexpr (ST == 1) asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
    else *p = v;
}

template <int LD, int ST>
__global__ __launch_bounds__(1024) void k_flat(const u32x4 *src, u32x4 *dst) {
    const long long i = (long long)blockIdx.x * 1024 + threadIdx.x;
    st<ST>(dst + i, sw(ld<LD>(src + i), 4));
}

// 128 short buffers of 2 MiB (128 blocks each) then 128 float buffers of 4 MiB (256 blocks each)
template <int LD, int ST>
__global__ __launch_bounds__(1024) void k_seg(const Seg *segs) {
    const long long b = blockIdx.x;
    const int s = b < 128 * 128 ? (int)(b / 128) : 128 + (int)((b - 128 * 128) / 256);
    const Seg sg = segs[s];
    const long long i = (b - sg.block0) * 1024 + threadIdx.x;
    st<ST>(sg.dst + i, sw(ld<LD>(sg.src + i), sg.es));
}

// persistent blocks with the next tile's load issued before the current
// tile's store (one 16 B vector per lane per tile, BS-lane tiles); tiles
// dealt round-robin over the grid (block k takes tiles k, k + grid, ...)
template <int BS, bool SEG>
__global__ __launch_bounds__(BS) void k_persist(const Seg *segs, const u32x4 *fsrc, u32x4 *fdst, long long ntile) {
    constexpr long long T2 = 2048 / BS * 128, T4 = 4096 / BS * 128;   // tiles per short / float buffer... per segment
    auto addr = [&](long long t, const u32x4 *&s, u32x4 *&d, int &es) {
        if constexpr (SEG) {
            const long long per_s = 2ll * (1 << 20) / (BS * 16), per_f = 4ll * (1 << 20) / (BS * 16);
            int k;
            long long rel;
            if (t < 128 * per_s) { k = (int)(t / per_s); rel = t - k * per_s; }
            else { const long long u = t - 128 * per_s; k = 128 + (int)(u / per_f); rel = u - (k - 128) * per_f; }
            s = segs[k].src + rel * BS + threadIdx.x;
            d = segs[k].dst + rel * BS + threadIdx.x;
            es = segs[k].es;
        } else {
            s = fsrc + t * BS + threadIdx.x;
            d = fdst + t * BS + threadIdx.x;
            es = 4;
        }
    };
    (void)T2; (void)T4;
    long long t = blockIdx.x;
    if (t >= ntile) return;
    const u32x4 *s; u32x4 *d; int es;
    addr(t, s, d, es);
    u32x4 v = __builtin_nontemporal_load(s);
    for (;;) {
        const long long tn = t + gridDim.x;
        const u32x4 *s2 = nullptr; u32x4 *d2 = nullptr; int es2 = 4;
        u32x4 v2;
        const bool more = tn < ntile;
        if (more) { addr(tn, s2, d2, es2); v2 = __builtin_nontemporal_load(s2); }
        st<1>(d, sw(v, es));
        if (!more) break;
        t = tn; d = d2; es = es2; v = v2;
    }
}

__global__ void k_rand(uint64_t *p, long long n, uint64_t seed) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main() {
    const long long total = 768ll << 20, nb = total / (1024 * 16);
    u32x4 *fs, *fd;
    CK(hipMalloc(&fs, total));
    CK(hipMalloc(&fd, total));
    k_rand<<<4096, 256>>>((uint64_t *)fs, total / 8, 1);
    std::vector<Seg> h(256);
    long long b0 = 0;
    for (int s = 0; s < 256; s++) {
        const int es = s < 128 ? 2 : 4;
        const size_t bytes = (size_t)es << 20;
        u32x4 *a, *d;
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&d, bytes));
        k_rand<<<1024, 256>>>((uint64_t *)a, (long long)bytes / 8, 100 + s);
        h[s] = {a, d, b0, es, 0};
        b0 += bytes / (1024 * 16);
    }
    if (b0 != nb) { printf("block count mismatch\n"); return 1; }
    Seg *ds;
    CK(hipMalloc(&ds, sizeof(Seg) * 256));
    CK(hipMemcpy(ds, h.data(), sizeof(Seg) * 256, hipMemcpyHostToDevice));
    struct V { std::string n; void (*f)(const Seg *, u32x4 *, u32x4 *, long long); std::vector<float> ms; };
    std::vector<V> vs;
#define FL(L, S) vs.push_back({std::string("flat ld") + (L ? "plain" : "nt") + " st" + (S == 0 ? "nt" : S == 1 ? "nt_sc1" : "plain"), \
        [](const Seg *, u32x4 *a, u32x4 *d, long long n) { k_flat<L, S><<<n, 1024>>>(a, d); }, {}});
#define SG(L, S) vs.push_back({std::string("seg  ld") + (L ? "plain" : "nt") + " st" + (S == 0 ? "nt" : S == 1 ? "nt_sc1" : "plain"), \
        [](const Seg *s, u32x4 *, u32x4 *, long long n) { k_seg<L, S><<<n, 1024>>>(s); }, {}});
    FL(0, 0) FL(0, 1) FL(0, 2) SG(0, 0) SG(0, 1) SG(0, 2) SG(1, 1)
#define PS(BS, SEGM, OCC) vs.push_back({std::string("persist bs") + #BS + (SEGM ? " seg" : " flat") + " occ" + #OCC, \
        [](const Seg *s, u32x4 *a, u32x4 *d, long long n) { \
            k_persist<BS, SEGM><<<256 * OCC, BS>>>(s, a, d, n * 1024 / BS); }, {}});
    PS(256, true, 8)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    for (int r = 0; r < 8; r++)
        for (auto &v : vs) {
            v.f(ds, fs, fd, nb);
            CK(hipEventRecord(e0));
            for (int k = 0; k < reps; k++) v.f(ds, fs, fd, nb);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) v.ms.push_back(ms / reps);
        }
    CK(hipGetLastError());
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
        printf("%-28s median %.4f ms  %.1f GB/s  (%.1f%%)  best %.1f%%\n", v.n.c_str(), med, 2.0 * total / med / 1e6,
               2.0 * total / med / 1e6 / 80.0, 2.0 * total / best / 1e6 / 80.0);
    }
    return 0;
}
