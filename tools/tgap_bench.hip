// Rate of the short-run gather (k_tgap's put direction, 4-bit gap-step map,
// 8-byte swap) as a standalone kernel, for A/B of its shape without
// rebuilding libpncx: U chunks per wave in flight, and plain or nontemporal
// loads of the user side.  Layout as tools/flex_bench.py short_runs: 2^23
// runs of 1..7 doubles, gaps 0..4, 8 copies (2^28 elements).
//   hipcc --offload-arch=gfx950 -O3 -o tools/tgap_bench tools/tgap_bench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);
    return v;
}

template <int U, bool NTL>
__global__ __launch_bounds__(256) void k_gather(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
                                                uint32_t tn, int64_t textent, const unsigned *toff,
                                                const unsigned char *nib) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 4 * U;
    for (uint32_t u0 = blockIdx.x * 4 * U; u0 < nunits; u0 += step) {
        uint64_t sv[U];
        int64_t ko[U];
        bool ok[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            const uint32_t c = u / nq, q = u - c * nq, r = q * 64 + lane, rc = r < tn ? r : tn - 1;
            ok[i] = okw && r < tn;
            ko[i] = (int64_t)c * tn + rc;
            const uint32_t b = nib[(int64_t)q * 32 + (lane >> 1)];
            const uint32_t g = wave_inclusive_sum((b >> ((lane & 1) * 4)) & 15u);
            const uint8_t *p = src + (int64_t)c * textent + toff[q] + (int64_t)((rc & 63) + g) * 8;
            if constexpr (NTL) sv[i] = __builtin_nontemporal_load((const uint64_t *)p);
            else sv[i] = *(const uint64_t *)p;
        }
#pragma unroll
        for (int i = 0; i < U; i++)
            if (ok[i]) __builtin_nontemporal_store(__builtin_bswap64(sv[i]), (uint64_t *)(dst + ko[i] * 8));
    }
}

// pairs: a lane moves elements 2p, 2p+1 of a 128-element pair of chunks
// (lanes 0-31 the first chunk, 32-63 the second), one 16-byte store; the
// gaps are a per-half prefix sum of the lane's two nibbles (one byte)
__device__ __forceinline__ uint32_t half_inclusive_sum(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);
    return v;
}
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
template <int U>
__global__ __launch_bounds__(256) void k_gather_pair(const uint8_t *src, uint8_t *dst, uint32_t npairs, uint32_t nq,
                                                     uint32_t tn, int64_t textent, const unsigned *toff,
                                                     const unsigned char *nib) {
    // requires tn % 128 == 0 here (the probe layout is trimmed to that)
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, lp = lane & 31;
    const uint32_t np = nq / 2;                       // pairs per copy
    const uint32_t step = gridDim.x * 4 * U;
    for (uint32_t u0 = blockIdx.x * 4 * U; u0 < npairs; u0 += step) {
        uint64_t a[U], b[U];
        int64_t ko[U];
        bool ok[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < npairs;
            u = __builtin_amdgcn_readfirstlane(okw ? u : npairs - 1);
            const uint32_t c = u / np, pr = u - c * np, q = 2 * pr + h;
            ok[i] = okw;
            const uint32_t by = nib[(int64_t)q * 32 + lp];
            const uint32_t n0 = by & 15u, n1 = by >> 4;
            const uint32_t P = half_inclusive_sum(n0 + n1);
            const uint8_t *base = src + (int64_t)c * textent + toff[q];
            const uint32_t e1 = 2 * lp + 1;
            a[i] = __builtin_nontemporal_load((const uint64_t *)(base + (int64_t)(e1 - 1 + P - n1) * 8));
            b[i] = __builtin_nontemporal_load((const uint64_t *)(base + (int64_t)(e1 + P) * 8));
            ko[i] = (int64_t)c * tn + (int64_t)q * 64 + 2 * lp;
        }
#pragma unroll
        for (int i = 0; i < U; i++)
            if (ok[i]) {
                u64x2 v = {__builtin_bswap64(a[i]), __builtin_bswap64(b[i])};
                __builtin_nontemporal_store(v, (u64x2 *)(dst + ko[i] * 8));
            }
    }
}

template <int U>
float run_pair(const uint8_t *s, uint8_t *d, uint32_t npairs, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
               const unsigned char *nb) {
    const unsigned grid = (npairs + 4 * U - 1) / (4 * U);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_gather_pair<U>), dim3(grid), dim3(256), 0, 0, s, d, npairs, nq, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_gather_pair<U>), dim3(grid), dim3(256), 0, 0, s, d, npairs, nq, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

// realign: the 4 waves of a block convert 4 consecutive chunks (256 packed
// elements when they lie in one copy); the values go through LDS and are
// stored from 64-element-aligned packed positions, so only the block's two
// edge lines are partial instead of every wave's
template <int U>
__global__ __launch_bounds__(256) void k_gather_realign(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
                                                        uint32_t tn, int64_t textent, const unsigned *toff,
                                                        const unsigned char *nib) {
    __shared__ uint64_t lv[U][256];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 4 * U;
    for (uint32_t u0 = blockIdx.x * 4 * U; u0 < nunits; u0 += step) {
        uint64_t sv[U];
        int64_t ko[U];
        bool ok[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            const uint32_t c = u / nq, q = u - c * nq, r = q * 64 + lane, rc = r < tn ? r : tn - 1;
            ok[i] = okw && r < tn;
            ko[i] = (int64_t)c * tn + rc;
            const uint32_t b = nib[(int64_t)q * 32 + (lane >> 1)];
            const uint32_t g = wave_inclusive_sum((b >> ((lane & 1) * 4)) & 15u);
            const uint8_t *p = src + (int64_t)c * textent + toff[q] + (int64_t)((rc & 63) + g) * 8;
            sv[i] = __builtin_nontemporal_load((const uint64_t *)p);
        }
#pragma unroll
        for (int i = 0; i < U; i++) {
            // the block's 4 chunks for this i: units ua..ua+3
            const uint32_t ua = u0 + i * 4;
            const uint32_t ca = ua / nq, qa = ua - ca * nq;
            const bool whole = ua + 3 < nunits && qa + 3 < nq && (qa + 4) * 64 <= tn;   // 4 full chunks, one copy
            if (whole) {
                lv[i][threadIdx.x] = __builtin_bswap64(sv[i]);
            } else if (ok[i]) {
                __builtin_nontemporal_store(__builtin_bswap64(sv[i]), (uint64_t *)(dst + ko[i] * 8));
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < U; i++) {
            const uint32_t ua = u0 + i * 4;
            const uint32_t ca = ua / nq, qa = ua - ca * nq;
            const bool whole = ua + 3 < nunits && qa + 3 < nq && (qa + 4) * 64 <= tn;
            if (!whole) continue;
            const int64_t p0 = (int64_t)ca * tn + (int64_t)qa * 64;      // first packed element of the 256
            const int64_t a0 = p0 & ~63LL;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int64_t k = a0 + threadIdx.x + 256 * j;
                if (k >= p0 && k < p0 + 256) __builtin_nontemporal_store(lv[i][k - p0], (uint64_t *)(dst + k * 8));
            }
        }
        __syncthreads();
    }
}

template <int U>
float run_ra(const uint8_t *s, uint8_t *d, uint32_t nunits, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
             const unsigned char *nb) {
    const unsigned grid = (nunits + 4 * U - 1) / (4 * U);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_gather_realign<U>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_gather_realign<U>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

// packed-aligned windows: wave = packed elements [64u, 64u + 64), which may
// span the tail of one map chunk, the next chunk and the next copy's first
// chunk (up to 3 segments, tn >= 64).  One wave scan over the lanes'
// nibbles gives the gaps inside each segment; the first segment also needs
// the gaps before its first position in its chunk: a second scan of that
// chunk's nibbles.  Stores are whole 512-byte runs at 64-element-aligned
// packed positions.
template <int U>
__global__ __launch_bounds__(256) void k_gather_win(const uint8_t *src, uint8_t *dst, uint32_t nwin, uint32_t n,
                                                    uint32_t tn, int64_t textent, const unsigned *toff,
                                                    const unsigned char *nib) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 4 * U;
    for (uint32_t u0 = blockIdx.x * 4 * U; u0 < nwin; u0 += step) {
        uint64_t sv[U];
        uint32_t kk[U];
        bool ok[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nwin;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nwin - 1);
            const uint32_t k0 = u * 64, c0 = k0 / tn, r0 = k0 - c0 * tn, q0 = r0 >> 6, p0 = r0 & 63;
            const uint32_t bc = (c0 + 1) * tn - k0;                     // lanes left in copy c0
            const uint32_t e0 = 64 - p0 < bc ? 64 - p0 : bc;            // end of segment 0
            const bool s1copy = e0 == bc;                               // segment 1 starts copy c0 + 1
            const uint32_t e1 = !s1copy && bc < 64 ? bc : 64;           // end of segment 1
            uint32_t c, q, pos;
            if (lane < e0) { c = c0; q = q0; pos = p0 + lane; }
            else if (lane < e1) { c = s1copy ? c0 + 1 : c0; q = s1copy ? 0 : q0 + 1; pos = lane - e0; }
            else { c = c0 + 1; q = 0; pos = lane - e1; }
            const uint32_t k = k0 + lane;
            ok[i] = okw && k < n;
            kk[i] = k;
            const uint32_t b = nib[(int64_t)q * 32 + (pos >> 1)];
            const uint32_t S = wave_inclusive_sum((b >> ((pos & 1) * 4)) & 15u);
            uint32_t m0 = 0;
            if (p0 != 0) {
                const uint32_t b0 = nib[(int64_t)q0 * 32 + (lane >> 1)];
                const uint32_t T = wave_inclusive_sum((b0 >> ((lane & 1) * 4)) & 15u);
                m0 = __builtin_amdgcn_readlane(T, p0 - 1);
            }
            const uint32_t s0 = __builtin_amdgcn_readlane(S, e0 - 1);
            const uint32_t s1 = __builtin_amdgcn_readlane(S, (e1 < 64 ? e1 : 64) - 1);
            const uint32_t g = lane < e0 ? m0 + S : lane < e1 ? S - s0 : S - s1;
            const uint8_t *p = ok[i] ? src + (int64_t)c * textent + toff[q] + (int64_t)(pos + g) * 8 : src;
            sv[i] = __builtin_nontemporal_load((const uint64_t *)p);
        }
#pragma unroll
        for (int i = 0; i < U; i++)
            if (ok[i]) __builtin_nontemporal_store(__builtin_bswap64(sv[i]), (uint64_t *)(dst + (int64_t)kk[i] * 8));
    }
}

template <int U>
float run_win(const uint8_t *s, uint8_t *d, uint32_t n, uint32_t tn, int64_t ext, const unsigned *t,
              const unsigned char *nb) {
    const uint32_t nwin = (n + 63) / 64;
    const unsigned grid = (nwin + 4 * U - 1) / (4 * U);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_gather_win<U>), dim3(grid), dim3(256), 0, 0, s, d, nwin, n, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_gather_win<U>), dim3(grid), dim3(256), 0, 0, s, d, nwin, n, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

// staged: every unit's map loads first, then the scans, then the element
// loads, then the stores (explicit software pipelining of the U units)
template <int U, int BS>
__global__ __launch_bounds__(BS) void k_gather_st(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
                                                  uint32_t tn, int64_t textent, const unsigned *toff,
                                                  const unsigned char *nib) {
    constexpr int W = BS / 64;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * W * U;
    for (uint32_t u0 = blockIdx.x * W * U; u0 < nunits; u0 += step) {
        uint32_t c[U], q[U], rc[U], b[U], tq[U];
        bool ok[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * W + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            c[i] = u / nq;
            q[i] = u - c[i] * nq;
            const uint32_t r = q[i] * 64 + lane;
            rc[i] = r < tn ? r : tn - 1;
            ok[i] = okw && r < tn;
            b[i] = nib[(int64_t)q[i] * 32 + (lane >> 1)];
            tq[i] = toff[q[i]];
        }
        uint64_t sv[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            const uint32_t g = wave_inclusive_sum((b[i] >> ((lane & 1) * 4)) & 15u);
            const uint8_t *p = src + (int64_t)c[i] * textent + tq[i] + (int64_t)((rc[i] & 63) + g) * 8;
            sv[i] = __builtin_nontemporal_load((const uint64_t *)p);
        }
#pragma unroll
        for (int i = 0; i < U; i++)
            if (ok[i])
                __builtin_nontemporal_store(__builtin_bswap64(sv[i]), (uint64_t *)(dst + ((int64_t)c[i] * tn + rc[i]) * 8));
    }
}

template <int U, int BS>
float run_st(const uint8_t *s, uint8_t *d, uint32_t nunits, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
             const unsigned char *nb) {
    const unsigned grid = (nunits + (BS / 64) * U - 1) / ((BS / 64) * U);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_gather_st<U, BS>), dim3(grid), dim3(BS), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_gather_st<U, BS>), dim3(grid), dim3(BS), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

// get direction: packed -> user scatter.  MODE 0: plain 8-byte stores at
// the user positions (k_tgap today); 1: nontemporal stores; 2: the chunk's
// user span loaded into LDS, the elements merged there, the span written
// back whole in 16-byte pieces (gap bytes rewritten with the values read)
template <int U, int MODE>
__global__ __launch_bounds__(256) void k_scatter(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
                                                 uint32_t tn, int64_t textent, const unsigned *toff,
                                                 const unsigned char *nib) {
    constexpr int SLOT = 3072;
    __shared__ __attribute__((aligned(16))) uint8_t lds[MODE == 2 ? 4 * U * SLOT : 16];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 4 * U;
    for (uint32_t u0 = blockIdx.x * 4 * U; u0 < nunits; u0 += step) {
        uint64_t sv[U];
        uint8_t *up[U];
        bool ok[U];
        uint32_t pos[U], last[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            const uint32_t c = u / nq, q = u - c * nq, r = q * 64 + lane, rc = r < tn ? r : tn - 1;
            ok[i] = okw && r < tn;
            const uint32_t b = nib[(int64_t)q * 32 + (lane >> 1)];
            const uint32_t g = wave_inclusive_sum((b >> ((lane & 1) * 4)) & 15u);
            pos[i] = (rc & 63) + g;
            last[i] = __builtin_amdgcn_readlane(pos[i], 63);
            up[i] = dst + (int64_t)c * textent + toff[q];
            sv[i] = __builtin_nontemporal_load((const uint64_t *)(src + ((int64_t)c * tn + rc) * 8));
            if (!okw) ok[i] = false;
        }
        if constexpr (MODE < 2) {
#pragma unroll
            for (int i = 0; i < U; i++) {
                if (!ok[i]) continue;
                uint64_t *p = (uint64_t *)(up[i] + pos[i] * 8);
                if constexpr (MODE == 1) __builtin_nontemporal_store(__builtin_bswap64(sv[i]), p);
                else *p = __builtin_bswap64(sv[i]);
            }
        } else {
#pragma unroll
            for (int i = 0; i < U; i++) {
                uint8_t *sl = lds + (w * U + i) * SLOT;
                const uint32_t bytes = (last[i] + 1) * 8;            // 8-aligned span from the chunk's first element
                for (uint32_t o = lane * 8; o < bytes; o += 512)
                    *(uint64_t *)(sl + o) = *(const uint64_t *)(up[i] + o);
            }
#pragma unroll
            for (int i = 0; i < U; i++) {
                uint8_t *sl = lds + (w * U + i) * SLOT;
                if (ok[i]) *(uint64_t *)(sl + pos[i] * 8) = __builtin_bswap64(sv[i]);
            }
#pragma unroll
            for (int i = 0; i < U; i++) {
                const uint8_t *sl = lds + (w * U + i) * SLOT;
                const uint32_t bytes = (last[i] + 1) * 8;
                for (uint32_t o = lane * 8; o < bytes; o += 512)
                    *(uint64_t *)(up[i] + o) = *(const uint64_t *)(sl + o);
            }
        }
    }
}

template <int U, int MODE>
float run_sc(const uint8_t *s, uint8_t *d, uint32_t nunits, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
             const unsigned char *nb) {
    const unsigned grid = (nunits + 4 * U - 1) / (4 * U);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_scatter<U, MODE>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_scatter<U, MODE>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

// the chunk's span read whole (16-byte pieces, contiguous per instruction)
// into LDS, then each lane picks its element from LDS
template <int U>
__global__ __launch_bounds__(256) void k_gather_lds(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
                                                    uint32_t tn, int64_t textent, const unsigned *toff,
                                                    const unsigned char *nib) {
    constexpr int SLOT = 3072;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * U * SLOT];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 4 * U;
    for (uint32_t u0 = blockIdx.x * 4 * U; u0 < nunits; u0 += step) {
        int64_t ko[U];
        bool ok[U];
        uint32_t pos[U];
        uint32_t lo16[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            const uint32_t c = u / nq, q = u - c * nq, r = q * 64 + lane, rc = r < tn ? r : tn - 1;
            ok[i] = okw && r < tn;
            ko[i] = (int64_t)c * tn + rc;
            const uint32_t b = nib[(int64_t)q * 32 + (lane >> 1)];
            const uint32_t g = wave_inclusive_sum((b >> ((lane & 1) * 4)) & 15u);
            const uint32_t last = __builtin_amdgcn_readlane(g + (rc & 63), 63);   // element offset of the last lane
            const uint8_t *base = src + (int64_t)c * textent + toff[q];
            const uintptr_t a0 = (uintptr_t)base & ~(uintptr_t)15;
            lo16[i] = (uint32_t)((uintptr_t)base - a0);
            const uint32_t bytes = lo16[i] + (last + 1) * 8;
            uint8_t *sl = lds + (w * U + i) * SLOT;
            for (uint32_t o = lane * 16; o < bytes; o += 1024)
                *(u32x4 *)(sl + o) = __builtin_nontemporal_load((const u32x4 *)(a0 + o));
            pos[i] = (rc & 63) + g;
        }
#pragma unroll
        for (int i = 0; i < U; i++) {
            const uint8_t *sl = lds + (w * U + i) * SLOT;
            uint64_t v;
            __builtin_memcpy(&v, sl + lo16[i] + pos[i] * 8, 8);
            if (ok[i]) __builtin_nontemporal_store(__builtin_bswap64(v), (uint64_t *)(dst + ko[i] * 8));
        }
    }
}

template <int U>
float run_lds(const uint8_t *s, uint8_t *d, uint32_t nunits, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
              const unsigned char *nb) {
    const unsigned grid = (nunits + 4 * U - 1) / (4 * U);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_gather_lds<U>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_gather_lds<U>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
    const uint32_t per = nb / 8, rem = nb % 8, x = b % 8, k = b / 8;
    return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
}

// store policy on the packed side: 0 nt (as k_gather), 1 plain write-back,
// 2 nt sc1 (st_stream in the library), with nontemporal user-side loads;
// round 5: 3 / 4 = the lanes whose 128-byte line the chunk covers only in
// part store write-back (the neighbouring chunk, usually a wave of the same
// block, fills the rest in L2 before it goes out whole), the others nt / nt sc1.
// Blocks in XCD order as k_tgap.
template <int U, int SP>
__global__ __launch_bounds__(256) void k_gather_sp(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
                                                   uint32_t tn, int64_t textent, const unsigned *toff,
                                                   const unsigned char *nib) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 4 * U;
    for (uint32_t u0 = xcd_remap(blockIdx.x, gridDim.x) * 4 * U; u0 < nunits; u0 += step) {
        uint64_t sv[U];
        int64_t ko[U];
        bool ok[U], edge[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            const uint32_t c = u / nq, q = u - c * nq, r = q * 64 + lane, rc = r < tn ? r : tn - 1;
            ok[i] = okw && r < tn;
            ko[i] = (int64_t)c * tn + rc;
            const int64_t lo = ((int64_t)c * tn + q * 64) * 8, hi = lo + (int64_t)(tn - q * 64 < 64 ? tn - q * 64 : 64) * 8;
            const int64_t line = (ko[i] * 8) & ~(int64_t)127;
            edge[i] = line < lo || line + 128 > hi;
            const uint32_t b = nib[(int64_t)q * 32 + (lane >> 1)];
            const uint32_t g = wave_inclusive_sum((b >> ((lane & 1) * 4)) & 15u);
            const uint8_t *p = src + (int64_t)c * textent + toff[q] + (int64_t)((rc & 63) + g) * 8;
            sv[i] = __builtin_nontemporal_load((const uint64_t *)p);
        }
#pragma unroll
        for (int i = 0; i < U; i++)
            if (ok[i]) {
                uint64_t *p = (uint64_t *)(dst + ko[i] * 8);
                const uint64_t v = __builtin_bswap64(sv[i]);
                if constexpr (SP == 0) __builtin_nontemporal_store(v, p);
                else if constexpr (SP == 1) *p = v;
                else if constexpr (SP == 2) asm volatile("global_store_dwordx2 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
                else if (edge[i]) *p = v;
                else if constexpr (SP == 3) __builtin_nontemporal_store(v, p);
                else asm volatile("global_store_dwordx2 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
            }
    }
}

template <int U, int SP>
float run_sp(const uint8_t *s, uint8_t *d, uint32_t nunits, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
             const unsigned char *nb) {
    const unsigned grid = (nunits + 4 * U - 1) / (4 * U);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_gather_sp<U, SP>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_gather_sp<U, SP>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

template <int U, bool NTL>
float run(const uint8_t *s, uint8_t *d, uint32_t nunits, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
          const unsigned char *nb, unsigned cap = 0) {
    unsigned grid = (nunits + 4 * U - 1) / (4 * U);
    if (cap && grid > cap) grid = cap;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((k_gather<U, NTL>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(a, 0);
    for (int k = 0; k < 20; k++)
        hipLaunchKernelGGL((k_gather<U, NTL>), dim3(grid), dim3(256), 0, 0, s, d, nunits, nq, tn, ext, t, nb);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

int main() {
    std::mt19937_64 g(5);
    const int nb = 1 << 23, copies = 8;
    std::vector<unsigned> o;
    o.reserve((size_t)nb * 4);
    unsigned long long pos = 0;
    for (int i = 0; i < nb; i++) {
        const int len = 1 + (int)(g() % 7), gap = (int)(g() % 5);
        for (int e = 0; e < len; e++) o.push_back((unsigned)((pos + e) * 8));
        pos += len + gap;
    }
    if (getenv("TRIM")) o.resize(o.size() / 128 * 128);   // whole chunk pairs (k_gather_pair)
    const uint32_t tn = (uint32_t)o.size(), nq = (tn + 63) / 64, nunits = nq * copies;
    const int64_t ext = (int64_t)pos * 8;
    std::vector<unsigned> base(nq);
    std::vector<unsigned char> nib(32 * (size_t)nq, 0);
    for (uint32_t e = 0; e < tn; e++) {
        if ((e & 63) == 0) { base[e >> 6] = o[e]; continue; }
        nib[e >> 1] |= (unsigned char)(((o[e] - o[e - 1]) / 8 - 1) << ((e & 1) * 4));
    }
    uint8_t *s, *d; unsigned *t; unsigned char *nbp;
    if (hipMalloc(&s, (size_t)ext * copies) || hipMalloc(&d, (size_t)tn * copies * 8) ||
        hipMalloc(&t, 4 * (size_t)nq) || hipMalloc(&nbp, nib.size())) return 4;
    hipMemset(s, 1, (size_t)ext * copies);
    hipMemcpy(t, base.data(), 4 * (size_t)nq, hipMemcpyHostToDevice);
    hipMemcpy(nbp, nib.data(), nib.size(), hipMemcpyHostToDevice);
    const double alg = (double)tn * copies * 16;
    // correctness of the LDS variant against the plain one
    {
        std::vector<uint8_t> hs((size_t)ext * copies);
        for (size_t i = 0; i < hs.size(); i++) hs[i] = (uint8_t)(i * 2654435761u >> 13);
        hipMemcpy(s, hs.data(), hs.size(), hipMemcpyHostToDevice);
        uint8_t *d2;
        if (hipMalloc(&d2, (size_t)tn * copies * 8)) return 4;
        run<4, false>(s, d, nunits, nq, tn, ext, t, nbp);
        run_sp<4, 1>(s, d2, nunits, nq, tn, ext, t, nbp);
        std::vector<uint8_t> h1((size_t)tn * copies * 8), h2(h1.size());
        hipMemcpy(h1.data(), d, h1.size(), hipMemcpyDeviceToHost);
        hipMemcpy(h2.data(), d2, h2.size(), hipMemcpyDeviceToHost);
        printf("write-back store variant %s the plain gather\n", h1 == h2 ? "matches" : "DIFFERS from");
        hipFree(d2);
    }
    {
        // scatter modes agree: the user buffer after MODE 0 and MODE 2 from
        // the same packed input and the same starting user bytes
        uint8_t *pk, *u1, *u2;
        const size_t ub = (size_t)ext * copies, pb = (size_t)tn * copies * 8;
        if (hipMalloc(&pk, pb) || hipMalloc(&u1, ub) || hipMalloc(&u2, ub)) return 4;
        std::vector<uint8_t> hp(pb), hu(ub);
        for (size_t i = 0; i < pb; i++) hp[i] = (uint8_t)(i * 2246822519u >> 11);
        for (size_t i = 0; i < ub; i++) hu[i] = (uint8_t)(i * 3266489917u >> 17);
        hipMemcpy(pk, hp.data(), pb, hipMemcpyHostToDevice);
        hipMemcpy(u1, hu.data(), ub, hipMemcpyHostToDevice);
        hipMemcpy(u2, hu.data(), ub, hipMemcpyHostToDevice);
        run_sc<4, 0>(pk, u1, nunits, nq, tn, ext, t, nbp);
        run_sc<2, 2>(pk, u2, nunits, nq, tn, ext, t, nbp);
        std::vector<uint8_t> h1(ub), h2(ub);
        hipMemcpy(h1.data(), u1, ub, hipMemcpyDeviceToHost);
        hipMemcpy(h2.data(), u2, ub, hipMemcpyDeviceToHost);
        printf("lds-merge scatter %s the plain scatter\n", h1 == h2 ? "matches" : "DIFFERS from");
        for (int rep = 0; rep < 0; rep++)
            printf("get: plain4 %.1f  nt4 %.1f  plain2 %.1f  lds1 %.1f  lds2 %.1f GB/s\n",
                   alg / run_sc<4, 0>(pk, u1, nunits, nq, tn, ext, t, nbp) / 1e6,
                   alg / run_sc<4, 1>(pk, u1, nunits, nq, tn, ext, t, nbp) / 1e6,
                   alg / run_sc<2, 0>(pk, u1, nunits, nq, tn, ext, t, nbp) / 1e6,
                   alg / run_sc<1, 2>(pk, u1, nunits, nq, tn, ext, t, nbp) / 1e6,
                   alg / run_sc<2, 2>(pk, u1, nunits, nq, tn, ext, t, nbp) / 1e6);
        hipFree(pk); hipFree(u1); hipFree(u2);
    }
    {
        // edge-line store variants write the same packed bytes as nt
        std::vector<uint8_t> h1((size_t)tn * copies * 8), h2(h1.size());
        hipMemset(d, 0, h1.size());
        run_sp<4, 0>(s, d, nunits, nq, tn, ext, t, nbp);
        hipMemcpy(h1.data(), d, h1.size(), hipMemcpyDeviceToHost);
        for (int m = 3; m <= 4; m++) {
            hipMemset(d, 0, h1.size());
            if (m == 3) run_sp<4, 3>(s, d, nunits, nq, tn, ext, t, nbp);
            else run_sp<4, 4>(s, d, nunits, nq, tn, ext, t, nbp);
            hipMemcpy(h2.data(), d, h2.size(), hipMemcpyDeviceToHost);
            printf("edge-line store variant %d %s nt\n", m, h1 == h2 ? "matches" : "DIFFERS from");
        }
    }
    for (int rep = 0; rep < 3; rep++)
        printf("tn %u (tn %% 64 = %u): store nt %.1f  write-back %.1f  nt sc1 %.1f  edge-wb+nt %.1f  edge-wb+nt-sc1 %.1f"
               " | U2: nt %.1f  wb %.1f GB/s\n", tn, tn % 64,
               alg / run_sp<4, 0>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_sp<4, 1>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_sp<4, 2>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_sp<4, 3>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_sp<4, 4>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_sp<2, 0>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_sp<2, 1>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6);
    for (int rep = 0; rep < 0; rep++)
        printf("U4nt grid cap: none %.1f  1024 %.1f  2048 %.1f  4096 %.1f  8192 %.1f  16384 %.1f  32768 %.1f GB/s\n",
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp, 1024) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp, 2048) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp, 4096) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp, 8192) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp, 16384) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp, 32768) / 1e6);
    for (int rep = 0; rep < 0; rep++) {
        printf("U4 %.1f  U4nt %.1f  st4x256 %.1f  st8x256 %.1f  st4x512 %.1f  st4x1024 %.1f  st2x1024 %.1f  st8x128 %.1f GB/s\n",
               alg / run<4, false>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_st<4, 256>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_st<8, 256>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_st<4, 512>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_st<4, 1024>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_st<2, 1024>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run_st<8, 128>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6);
    }
    return 0;
}
