// c4_shape_sweep.hip -- block shape and block order for the C4 swap batch.
// Standalone; not part of the product.  The product's flat 4-byte swap
// (k_tile: 256 lanes, XCD-contiguous block order) moves the C4 batch's
// bytes (768 MiB -> 768 MiB, one buffer pair) at 83.6 % of peak back to back
// (tools/oop_probe.py), while k_batch_swapmix (1024 lanes, launch order)
// moves them over the 256 variables at 79.4 %.  This sweep separates the two
// differences on the C4 layout (256 hipMalloc buffer pairs, 2 / 4 MiB
// alternating by class, splitmix64 data), one 16 B vector per lane, nt loads,
// "nt sc1" stores:
//   flat|seg  L lanes  remap 0|1
// remap = XCD-contiguous tile order (the bijective formula of k_tile).
// Launches queued back to back (20 per sample); interleaved rounds.
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

__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ long long remap(long long b, long long nb) {
    const long long q = nb >> 3, r = nb & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

template <int L, bool RM>
__global__ __launch_bounds__(L) void k_flat(const u32x4 *src, u32x4 *dst) {
    const long long t = RM ? remap(blockIdx.x, gridDim.x) : (long long)blockIdx.x;
    const long long i = t * L + threadIdx.x;
    st(dst + i, sw(__builtin_nontemporal_load(src + i), 4));
}

// 128 short buffers of 2 MiB then 128 float buffers of 4 MiB (the product's
// group rule: segment = s0 + (t - b0) / per)
template <int L, bool RM>
__global__ __launch_bounds__(L) void k_seg(const Seg *segs) {
    constexpr long long PS = (2ll << 20) / (L * 16), PF = (4ll << 20) / (L * 16);
    const long long t = RM ? remap(blockIdx.x, gridDim.x) : (long long)blockIdx.x;
    const int s = t < 128 * PS ? (int)(t / PS) : 128 + (int)((t - 128 * PS) / PF);
    const Seg sg = segs[s];
    const long long i = (t - sg.block0) * L + threadIdx.x;
    st(sg.dst + i, sw(__builtin_nontemporal_load(sg.src + i), sg.es));
}

// translation warm-up: the first block of each segment has one lane load a
// word from every 2 MiB of the segment D ahead (source and destination), so
// a TLB miss there is taken before that segment's blocks need it
template <int L, int D>
__global__ __launch_bounds__(L) void k_segt(const Seg *segs) {
    constexpr long long PS = (2ll << 20) / (L * 16), PF = (4ll << 20) / (L * 16);
    const long long t = remap(blockIdx.x, gridDim.x);
    const int s = t < 128 * PS ? (int)(t / PS) : 128 + (int)((t - 128 * PS) / PF);
    const Seg sg = segs[s];
    const long long rel = t - sg.block0;
    if (rel == 0 && threadIdx.x < 4 && s + D < 256) {
        const Seg nx = segs[s + D];
        const char *p = (threadIdx.x & 1) ? (const char *)nx.dst : (const char *)nx.src;
        p += (threadIdx.x >> 1) * (2 << 20);
        if ((threadIdx.x >> 1) * 2 < nx.es) {
            unsigned w = __builtin_nontemporal_load((const unsigned *)p);
            asm volatile("" ::"v"(w));
        }
    }
    const long long i = rel * L + threadIdx.x;
    st(sg.dst + i, sw(__builtin_nontemporal_load(sg.src + i), sg.es));
}

// U vectors per lane (tile = L x 16 x U bytes, each instruction one
// contiguous L x 16 B run), all loads issued before the stores: the
// descriptor's dependent load is paid once per U vectors
template <int L, int U, bool SEG>
__global__ __launch_bounds__(L) void k_segu(const Seg *segs, const u32x4 *fsrc, u32x4 *fdst) {
    constexpr long long PS = (2ll << 20) / (L * 16 * U), PF = (4ll << 20) / (L * 16 * U);
    const long long t = remap(blockIdx.x, gridDim.x);
    const u32x4 *src;
    u32x4 *dst;
    int es = 4;
    if constexpr (SEG) {
        const int s = t < 128 * PS ? (int)(t / PS) : 128 + (int)((t - 128 * PS) / PF);
        const Seg sg = segs[s];
        const long long rel = t - (s < 128 ? s * PS : 128 * PS + (s - 128) * PF);
        src = sg.src + rel * L * U;
        dst = sg.dst + rel * L * U;
        es = sg.es;
    } else {
        src = fsrc + t * L * U;
        dst = fdst + t * L * U;
    }
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(src + u * L + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; u++) st(dst + u * L + threadIdx.x, sw(v[u], es));
}

__global__ void k_rand(uint64_t *p, long long n, uint64_t seed) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

struct V { std::string n; int lanes; int u; int pool; void (*f)(const Seg *, const u32x4 *, u32x4 *, long long); std::vector<float> ms; };

int main() {
    const long long total = 768ll << 20;
    u32x4 *fs, *fd;
    CK(hipMalloc(&fs, total));
    CK(hipMalloc(&fd, total));
    k_rand<<<4096, 256>>>((uint64_t *)fs, total / 8, 1);
    // descriptor tables per lane count (block0 in tiles of L lanes)
    std::vector<Seg> h(256);
    for (int s = 0; s < 256; s++) {
        const int es = s < 128 ? 2 : 4;
        const size_t bytes = (size_t)es << 20;
        u32x4 *a, *d;
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&d, bytes));
        k_rand<<<1024, 256>>>((uint64_t *)a, (long long)bytes / 8, 100 + s);
        h[s] = {a, d, 0, es, 0};
    }
    // tables 0-2: the 256 separate buffer pairs; 3-5: the same descriptors
    // pointing into the flat pair (one allocation per side, "pool")
    Seg *dsegs[6];
    const int lanes[3] = {256, 512, 1024};
    std::vector<Seg> sep = h;
    for (int k = 0; k < 6; k++) {
        long long b0 = 0;
        size_t off = 0;
        for (int s = 0; s < 256; s++) {
            h[s] = sep[s];
            if (k >= 3) {
                h[s].src = (const u32x4 *)((const char *)fs + off);
                h[s].dst = (u32x4 *)((char *)fd + off);
            }
            off += (size_t)h[s].es << 20;
            h[s].block0 = b0;
            b0 += ((size_t)h[s].es << 20) / (lanes[k % 3] * 16);
        }
        if (b0 != total / (lanes[k % 3] * 16)) { printf("block count mismatch\n"); return 1; }
        CK(hipMalloc(&dsegs[k], sizeof(Seg) * 256));
        CK(hipMemcpy(dsegs[k], h.data(), sizeof(Seg) * 256, hipMemcpyHostToDevice));
    }
    std::vector<V> vs;
#define FL(L, RM) vs.push_back({"flat " #L " remap " #RM, L, 1, 0, [](const Seg *, const u32x4 *a, u32x4 *d, long long nb) { \
        k_flat<L, RM><<<nb, L>>>(a, d); }, {}});
#define SG(L, RM) vs.push_back({"seg  " #L " remap " #RM, L, 1, 0, [](const Seg *s, const u32x4 *, u32x4 *, long long nb) { \
        k_seg<L, RM><<<nb, L>>>(s); }, {}});
#define SU(L, U, SEGM) vs.push_back({std::string(SEGM ? "seg  " : "flat ") + #L " remap 1 U" #U, L, U, 0, \
        [](const Seg *s, const u32x4 *a, u32x4 *d, long long nb) { k_segu<L, U, SEGM><<<nb, L>>>(s, a, d); }, {}});
    FL(256, true) FL(1024, true) FL(1024, false)
    SG(256, true) SG(512, true) SG(1024, true) SG(1024, false)
    SU(256, 2, false)
    SU(256, 2, true)
#define PL(L, RM) vs.push_back({"pool " #L " remap " #RM, L, 1, 1, [](const Seg *s, const u32x4 *, u32x4 *, long long nb) { \
        k_seg<L, RM><<<nb, L>>>(s); }, {}});
    PL(256, true) PL(1024, true) PL(1024, false)
#define ST(L, D) vs.push_back({"seg  " #L " remap 1 touch" #D, L, 1, 0, [](const Seg *s, const u32x4 *, u32x4 *, long long nb) { \
        k_segt<L, D><<<nb, L>>>(s); }, {}});
    ST(256, 1) ST(256, 2) ST(1024, 1) ST(1024, 2)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    for (int r = 0; r < 9; r++)
        for (auto &v : vs) {
            const long long nb = total / (v.lanes * 16 * v.u);
            const Seg *ds = dsegs[(v.lanes == 256 ? 0 : v.lanes == 512 ? 1 : 2) + 3 * v.pool];
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
        printf("%-22s median %.4f ms  %.1f GB/s  (%.1f%%)  best %.1f%%\n", v.n.c_str(), med, 2.0 * total / med / 1e6,
               2.0 * total / med / 1e6 / 80.0, 2.0 * total / best / 1e6 / 80.0);
    }
    return 0;
}
