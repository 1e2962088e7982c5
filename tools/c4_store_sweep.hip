// c4_store_sweep.hip -- load/store cache policy for the C4-sized swap batch.
// Standalone; not part of the product.  768 MiB out-of-place 4-byte swap
// (1.5 GiB moved, the C4 batch's bytes) as one flat buffer pair and as 256
// buffers (2/4 MiB alternating, one hipMalloc each, block -> buffer by the
// group rule of k_batch_swapmix), 1024 lanes x 16 B per block, with
//   loads:  nt (nontemporal builtin) | plain
//   stores: nt | nt sc1 (inline asm) | plain
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

int main() {
    const long long total = 768ll << 20, nb = total / (1024 * 16);
    u32x4 *fs, *fd;
    CK(hipMalloc(&fs, total));
    CK(hipMalloc(&fd, total));
    CK(hipMemset(fs, 0x3c, total));
    std::vector<Seg> h(256);
    long long b0 = 0;
    for (int s = 0; s < 256; s++) {
        const int es = s < 128 ? 2 : 4;
        const size_t bytes = (size_t)es << 20;
        u32x4 *a, *d;
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&d, bytes));
        CK(hipMemset(a, 0x3c, bytes));
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
    FL(0, 0) FL(0, 1) FL(0, 2) FL(1, 0) FL(1, 1) FL(1, 2)
    SG(0, 0) SG(0, 1) SG(0, 2) SG(1, 0) SG(1, 1) SG(1, 2)
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
