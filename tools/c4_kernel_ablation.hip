// c4_kernel_ablation.hip -- where does the product's same-type batch kernel
// (k_batch_swapmix) lose to the minimal segmented kernel of
// tools/c4_shape_sweep.hip?  On one box the product ran the C4 bytes laid out
// as one pool per side at 81.3 % of peak and the minimal kernel at 84.2 %.
// Standalone; not part of the product.  Uses the product's own device code
// (pncx_kern.hpp: pncxk_seg, batch_segment, batch_block, ld16/st16), the C4
// layout as sub-ranges of one allocation per side ("pool") and as 256
// separate hipMalloc pairs ("sep"), splitmix64 data, 20 launches back to back
// per sample, interleaved rounds.
//   P0  the product kernel body (group lookup, descriptor, head/tail block,
//       4-way element-size switch)
//   P1  P0 without the head/tail block (the C4 segments have none)
//       (P0/P1 ran at 80.8 % on the pool with round 2's 8-run table read
//       whole; P6 83.5 %, P3 83.6 %: the product now reads one or two run
//       records, profiles/r02s_c4_ablation*.txt)
//   P2  P1 with the sweep's 2-way swap (es 2 or 4)
//   P3  P1 with the segment found by constant divisors (the sweep's rule)
//   P4  P1 reading only src/dst/aux/block0 (no head/nvec offsets)
//   P5  P1 with the run table read from device memory instead of the kernarg
//   P6  P1 with two runs passed as a compact kernarg struct
//   P7  P1 with the segment read from a device block -> segment map
//   MIN the minimal kernel (tools/c4_shape_sweep.hip k_seg<1024, remap>)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <string>
#include <vector>

#include "../pnetcdf_amd/csrc/pncx_kern.hpp"

using namespace pncx;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int L = 1024;

__device__ __forceinline__ u32x4 swap16(u32x4 v, int es) {    // the product's (pncx_kern_swap.hip)
    u32x4 r = v;
    if (es == 2) {
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = ((v[k] & 0x00ff00ffu) << 8) | ((v[k] >> 8) & 0x00ff00ffu);
    } else if (es == 4) {
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = __builtin_bswap32(v[k]);
    } else if (es == 8) {
        r[0] = __builtin_bswap32(v[1]); r[1] = __builtin_bswap32(v[0]);
        r[2] = __builtin_bswap32(v[3]); r[3] = __builtin_bswap32(v[2]);
    }
    return r;
}
__device__ __forceinline__ u32x4 swap16_2way(u32x4 v, int es) {
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

template <int ES>
__device__ __forceinline__ void mix_scalar(const uint8_t *src, uint8_t *dst, int64_t e0, int64_t e1) {
    using Op = SwapOp<ES>;
    bool bad = false;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += L) scalar_elem<Op>(src, dst, e, 0, bad);
}

struct Grp2 { int n, s01; long long b01; unsigned long long mag0, mag1; int shr0, shr1; };

template <int V>
__global__ __launch_bounds__(L) void k_var(const pncxk_seg *segs, int nseg, const int *map, pncxk_groups grp,
                                           const pncxk_groups *dgrp, Grp2 g2) {
    const long long b = batch_block();
    int s;
    if constexpr (V == 5) {
        s = batch_segment<false>(b, nullptr, *dgrp, segs, nseg);
    } else if constexpr (V == 6) {
        const bool hi = g2.n > 1 && b >= g2.b01;
        const unsigned long long r = (unsigned long long)(b - (hi ? g2.b01 : 0));
        s = (hi ? g2.s01 : 0) + (int)((r * (hi ? g2.mag1 : g2.mag0)) >> (hi ? g2.shr1 : g2.shr0));
    } else if constexpr (V == 7) {
        s = map[b];
    } else if constexpr (V == 3) {
        constexpr long long PS = (2ll << 20) / (L * 16), PF = (4ll << 20) / (L * 16);
        s = b < 128 * PS ? (int)(b / PS) : 128 + (int)((b - 128 * PS) / PF);
    } else {
        s = batch_segment<false>(b, map, grp, segs, nseg);
    }
    const pncxk_seg sg = segs[s];
    const uint8_t *src = (const uint8_t *)sg.src;
    uint8_t *dst = (uint8_t *)sg.dst;
    const int es = sg.aux;
    const int64_t rel = b - sg.block0;
    if constexpr (V == 4) {
        const int64_t off = (rel * L + threadIdx.x) * 16;
        st16<true>(dst + off, swap16(ld16<true>(src + off), es));
        return;
    }
    if (rel < sg.nvec) {
        const int64_t off = sg.head * es + (rel * L + threadIdx.x) * 16;
        if constexpr (V == 2) st16<true>(dst + off, swap16_2way(ld16<true>(src + off), es));
        else st16<true>(dst + off, swap16(ld16<true>(src + off), es));
    }
    if constexpr (V == 0) {
        if (rel == 0) {
            const int64_t tail0 = sg.head + sg.nvec * (int64_t)(L * 16 / es);
            switch (es) {
                case 1: mix_scalar<1>(src, dst, 0, sg.head); mix_scalar<1>(src, dst, tail0, sg.n); break;
                case 2: mix_scalar<2>(src, dst, 0, sg.head); mix_scalar<2>(src, dst, tail0, sg.n); break;
                case 4: mix_scalar<4>(src, dst, 0, sg.head); mix_scalar<4>(src, dst, tail0, sg.n); break;
                case 8: mix_scalar<8>(src, dst, 0, sg.head); mix_scalar<8>(src, dst, tail0, sg.n); break;
                default: break;
            }
        }
    }
}

struct MinSeg { const u32x4 *src; u32x4 *dst; long long block0; int es; int pad; };
__global__ __launch_bounds__(L) void k_min(const MinSeg *segs) {
    constexpr long long PS = (2ll << 20) / (L * 16), PF = (4ll << 20) / (L * 16);
    const long long t = xcd_remap(blockIdx.x, gridDim.x);
    const int s = t < 128 * PS ? (int)(t / PS) : 128 + (int)((t - 128 * PS) / PF);
    const MinSeg sg = segs[s];
    const long long i = (t - sg.block0) * L + threadIdx.x;
    st16<true>((uint8_t *)(sg.dst + i), swap16_2way(__builtin_nontemporal_load(sg.src + i), sg.es));
}

__global__ void k_rand(uint64_t *p, long long n, uint64_t seed) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        uint64_t z = seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

static void magic(pncxk_groups *g, int k) {       // the host rule of pncx_host.c group_magic
    int l = 0;
    while ((1LL << l) < g->r[k].per) l++;
    g->r[k].shr = 31 + l;
    g->r[k].mag = ((1ULL << g->r[k].shr) - 1) / (unsigned long long)g->r[k].per + 1;
}

int main() {
    const long long total = 768ll << 20, nb = total / (L * 16);
    uint8_t *ps, *pd;
    CK(hipMalloc(&ps, total));
    CK(hipMalloc(&pd, total));
    k_rand<<<4096, 256>>>((uint64_t *)ps, total / 8, 1);
    std::vector<pncxk_seg> hs[2];
    std::vector<MinSeg> hm[2];
    for (int lay = 0; lay < 2; lay++) {           // 0 pool, 1 sep
        long long b0 = 0, off = 0;
        for (int s = 0; s < 256; s++) {
            const int es = s < 128 ? 2 : 4;
            const long long bytes = (long long)es << 20;
            uint8_t *a = ps + off, *d = pd + off;
            if (lay == 1) {
                CK(hipMalloc(&a, bytes));
                CK(hipMalloc(&d, bytes));
                k_rand<<<1024, 256>>>((uint64_t *)a, bytes / 8, 100 + s);
            }
            pncxk_seg g{};
            g.src = a; g.dst = d; g.n = 1 << 20; g.head = 0; g.nvec = bytes / (L * 16); g.block0 = b0;
            g.fill = 0; g.status = nullptr; g.aux = es;
            hs[lay].push_back(g);
            hm[lay].push_back({(const u32x4 *)a, (u32x4 *)d, b0, es, 0});
            b0 += g.nvec;
            off += bytes;
        }
        if (b0 != nb) { printf("block count mismatch\n"); return 1; }
    }
    pncxk_groups grp{};
    grp.n = 2;
    grp.r[0].s0 = 0; grp.r[0].b0 = 0; grp.r[0].per = (2ll << 20) / (L * 16);
    grp.r[1].s0 = 128; grp.r[1].b0 = 128 * grp.r[0].per; grp.r[1].per = (4ll << 20) / (L * 16);
    magic(&grp, 0);
    magic(&grp, 1);
    pncxk_groups *dgrp;
    CK(hipMalloc(&dgrp, sizeof grp));
    CK(hipMemcpy(dgrp, &grp, sizeof grp, hipMemcpyHostToDevice));
    Grp2 g2{2, 128, grp.r[1].b0, grp.r[0].mag, grp.r[1].mag, grp.r[0].shr, grp.r[1].shr};
    std::vector<int> hmap(nb);
    for (long long b = 0; b < nb; b++)
        hmap[b] = b < grp.r[1].b0 ? (int)(b / grp.r[0].per) : 128 + (int)((b - grp.r[1].b0) / grp.r[0 + 1].per);
    int *dmap;
    CK(hipMalloc(&dmap, sizeof(int) * nb));
    CK(hipMemcpy(dmap, hmap.data(), sizeof(int) * nb, hipMemcpyHostToDevice));
    pncxk_seg *ds[2];
    MinSeg *dm[2];
    for (int lay = 0; lay < 2; lay++) {
        CK(hipMalloc(&ds[lay], sizeof(pncxk_seg) * 256));
        CK(hipMemcpy(ds[lay], hs[lay].data(), sizeof(pncxk_seg) * 256, hipMemcpyHostToDevice));
        CK(hipMalloc(&dm[lay], sizeof(MinSeg) * 256));
        CK(hipMemcpy(dm[lay], hm[lay].data(), sizeof(MinSeg) * 256, hipMemcpyHostToDevice));
    }
    struct Var { std::string n; int lay; int v; std::vector<float> ms; };
    std::vector<Var> vs;
    const char *names[] = {"P0", "P1", "P2", "P3", "P4", "P5", "P6", "P7", "MIN"};
    for (int lay = 0; lay < 2; lay++)
        for (int v = 0; v < 9; v++) vs.push_back({std::string(lay ? "sep  " : "pool ") + names[v], lay, v, {}});
    auto run = [&](const Var &v) {
        const pncxk_seg *s = ds[v.lay];
        switch (v.v) {
            case 0: k_var<0><<<nb, L>>>(s, 256, nullptr, grp, dgrp, g2); break;
            case 1: k_var<1><<<nb, L>>>(s, 256, nullptr, grp, dgrp, g2); break;
            case 2: k_var<2><<<nb, L>>>(s, 256, nullptr, grp, dgrp, g2); break;
            case 3: k_var<3><<<nb, L>>>(s, 256, nullptr, grp, dgrp, g2); break;
            case 4: k_var<4><<<nb, L>>>(s, 256, nullptr, grp, dgrp, g2); break;
            case 5: k_var<5><<<nb, L>>>(s, 256, nullptr, grp, dgrp, g2); break;
            case 6: k_var<6><<<nb, L>>>(s, 256, nullptr, grp, dgrp, g2); break;
            case 7: k_var<7><<<nb, L>>>(s, 256, dmap, grp, dgrp, g2); break;
            default: k_min<<<nb, L>>>(dm[v.lay]); break;
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    for (int r = 0; r < 9; r++)
        for (auto &v : vs) {
            run(v);
            CK(hipEventRecord(e0));
            for (int k = 0; k < reps; k++) run(v);
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
        printf("%-10s median %.4f ms  %.1f GB/s  (%.1f%%)  best %.1f%%\n", v.n.c_str(), med, 2.0 * total / med / 1e6,
               2.0 * total / med / 1e6 / 80.0, 2.0 * total / best / 1e6 / 80.0);
    }
    return 0;
}
