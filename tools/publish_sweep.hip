// publish_sweep.hip -- how a batch kernel should report "some element was
// out of range" (NC_ERANGE) per segment.  Standalone; not part of the
// product.  Workload: config 4's secondary variant, 128 segments x 2^20
// float -> NC_SHORT (16 B loads x2, 16 B store per lane, 2048 elements per
// block), values uniform in [-40000, 40000] (~18% out of range), a fresh
// status value every launch (as every synchronous pncx_dev_batch call and
// every host putn has).  Interleaved rounds in one process.
//   V0 per-wave ballot, agent-scope atomic load, store if different (round 1)
//   V1 per-block OR (LDS), one lane: atomic load, store if different
//   V2 per-wave ballot, plain (L2-cached) load, atomic store if different
//   V3 per-block flag word (plain store of the epoch, no sharing) + a
//      reduce kernel per call
//   V4 per-wave, status replicated per XCD (blockIdx & 7), atomic load/store
//   V5 no status (bandwidth reference)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int NSEG = 128, NEL = 1 << 20, TILE = 2048, BPS = NEL / TILE;

__device__ __forceinline__ uint32_t cvt2(float a, float b, bool &bad) {
    const bool ba = !(a <= 32767.0f && a >= -32768.0f), bb = !(b <= 32767.0f && b >= -32768.0f);
    bad |= ba | bb;
    const uint32_t x = ba ? 0x8001u : (uint32_t)(uint16_t)(int16_t)(int)a;
    const uint32_t y = bb ? 0x8001u : (uint32_t)(uint16_t)(int16_t)(int)b;
    const uint32_t sx = ((x & 0xff) << 8) | (x >> 8), sy = ((y & 0xff) << 8) | (y >> 8);
    return sx | (sy << 16);
}

__device__ __forceinline__ bool body(const float *src, short *dst, int64_t b) {
    const int seg = (int)(b / BPS), rel = (int)(b % BPS);
    const f32x4 *s = (const f32x4 *)(src + (int64_t)seg * NEL + (int64_t)rel * TILE) + threadIdx.x * 2;
    u32x4 *d = (u32x4 *)(dst + (int64_t)seg * NEL + (int64_t)rel * TILE) + threadIdx.x;
    const f32x4 v0 = __builtin_nontemporal_load(s), v1 = __builtin_nontemporal_load(s + 1);
    bool bad = false;
    u32x4 o;
    o.x = cvt2(v0.x, v0.y, bad);
    o.y = cvt2(v0.z, v0.w, bad);
    o.z = cvt2(v1.x, v1.y, bad);
    o.w = cvt2(v1.z, v1.w, bad);
    __builtin_nontemporal_store(o, d);
    return bad;
}

template <int V>
__global__ __launch_bounds__(256) void k_conv(const float *src, short *dst, int *status, int *flags, int sval) {
    const int64_t b = blockIdx.x;
    const int seg = (int)(b / BPS);
    const bool bad = body(src, dst, b);
    if constexpr (V == 0 || V == 2 || V == 4) {
        const unsigned long long m = __ballot(bad);
        int *st = V == 4 ? status + seg * 8 + (blockIdx.x & 7) : status + seg;
        if (m != 0 && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1)) {
            int cur;
            if constexpr (V == 2) cur = *(volatile int *)st;
            else cur = __hip_atomic_load(st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur != sval) __hip_atomic_store(st, sval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if constexpr (V == 1) {
        const int any = __syncthreads_or(bad);
        if (any && threadIdx.x == 0 &&
            __hip_atomic_load(status + seg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != sval)
            __hip_atomic_store(status + seg, sval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (V == 3) {
        const int any = __syncthreads_or(bad);
        if (any && threadIdx.x == 0) flags[b] = sval;
    }
}

// V3's reduce: one block per segment scans its blocks' flags
__global__ __launch_bounds__(256) void k_reduce(const int *flags, int *status, int sval) {
    const int seg = blockIdx.x;
    bool hit = false;
    for (int i = threadIdx.x; i < BPS; i += 256) hit |= flags[seg * BPS + i] == sval;
    if (__syncthreads_or(hit) && threadIdx.x == 0) status[seg] = sval;
}

int main()
{
    const size_t n = (size_t)NSEG * NEL;
    float *src;
    short *dst;
    int *status, *flags;
    CK(hipMalloc(&src, n * 4));
    CK(hipMalloc(&dst, n * 2));
    CK(hipMalloc(&status, NSEG * 8 * 4));
    CK(hipMalloc(&flags, (size_t)NSEG * BPS * 4));
    CK(hipMemset(status, 0, NSEG * 8 * 4));
    CK(hipMemset(flags, 0, (size_t)NSEG * BPS * 4));
    std::vector<float> h(n);
    uint64_t z = 0x5EED0004;
    for (size_t i = 0; i < n; i++) {
        z = z * 6364136223846793005ULL + 1442695040888963407ULL;
        h[i] = -40000.0f + 80000.0f * (float)((z >> 40) & 0xFFFFFF) / 16777216.0f;
    }
    CK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nb = NSEG * BPS, reps = 20;
    double tot[6] = {0};
    int sval = 1;
    for (int round = 0; round < 5; round++)
        for (int v = 0; v < 6; v++) {
            for (int r = 0; r < reps + 2; r++) {
                sval++;
                if (r == 2) CK(hipEventRecord(e0));
                switch (v) {
                case 0: k_conv<0><<<nb, 256>>>(src, dst, status, flags, sval); break;
                case 1: k_conv<1><<<nb, 256>>>(src, dst, status, flags, sval); break;
                case 2: k_conv<2><<<nb, 256>>>(src, dst, status, flags, sval); break;
                case 3: k_conv<3><<<nb, 256>>>(src, dst, status, flags, sval);
                        k_reduce<<<NSEG, 256>>>(flags, status, sval); break;
                case 4: k_conv<4><<<nb, 256>>>(src, dst, status, flags, sval); break;
                default: k_conv<5><<<nb, 256>>>(src, dst, status, flags, sval); break;
                }
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (round > 0) tot[v] += ms / reps;
            /* every segment must report (18% out of range in each) */
            std::vector<int> hs(NSEG * 8);
            CK(hipMemcpy(hs.data(), status, NSEG * 8 * 4, hipMemcpyDeviceToHost));
            if (v != 5)
                for (int s = 0; s < NSEG; s++) {
                    bool ok = v == 4 ? false : hs[s] == sval;
                    if (v == 4) for (int x = 0; x < 8; x++) ok |= hs[s * 8 + x] == sval;
                    if (!ok) { printf("V%d: segment %d status missing\n", v, s); return 1; }
                }
        }
    const double bytes = (double)n * 6;
    for (int v = 0; v < 6; v++)
        printf("V%d  %.4f ms  %.1f GB/s  (%.1f%% of 8 TB/s)\n", v, tot[v] / 4, bytes / (tot[v] / 4 * 1e-3) / 1e9,
               bytes / (tot[v] / 4 * 1e-3) / 8e12 * 100);
    return 0;
}
