// transpose_sweep.hip -- standalone tuning sweep for the varm transpose
// (k_imap_tile): a Fortran-order user buffer of doubles, count {C0, C1, C2}
// with imap {1, C0, C0*C1}, packed (C order) with an 8-byte swap.
//   user  element (u, o, p) at u + o*C0 + p*C0*C1      (U = dim 0, outer = dim 1, P = dim 2)
//   packed element (u, o, p) at u*C1*C2 + o*C2 + p
// Not part of the product; the winner is folded into pnetcdf_amd/csrc/
// pncx_kern.hpp.  Interleaved rounds in one process.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <string>
#include <functional>
#include <string.h>

#include "../pnetcdf_amd/csrc/pncx_kern.hpp"   // the product's k_imap_tile, same process

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint64_t u64;
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u64 sw8(u64 v) { return __builtin_bswap64(v); }

struct Geo { long long c0, c1, c2; };

// Tile TP (along P) x TU (along U); VU elements per lane on the user side
// (lanes along U), VP per lane on the packed side (lanes along P).
// OB outer indices per block (the same u/p tile for OB consecutive o).
template <int TP, int TU, int VU, int VP, int BS>
__global__ __launch_bounds__(BS) void k_tr(const u64 *user, u64 *packed, Geo g) {
    __shared__ u64 tile[TP][TU + 1];
    const long long ntu = g.c0 / TU, ntp = g.c2 / TP;
    long long b = blockIdx.x;
    const long long tu = b % ntu; b /= ntu;
    const long long tp = b % ntp; b /= ntp;
    const long long o = b;
    const long long u0 = tu * TU, p0 = tp * TP;
    // read: rows p (TP of them), each TU contiguous user elements; a row takes TU/VU lanes
    constexpr int LPR = TU / VU;                  // lanes per row
    constexpr int RPP = BS / LPR;                 // rows per pass
    constexpr int NR = TP / RPP;                  // passes
    const int t = threadIdx.x;
    {
        const int lr = t % LPR, r0 = t / LPR;
        u64 v[NR][VU];
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const long long p = p0 + r0 + i * RPP;
            const u64 *src = user + u0 + lr * VU + o * g.c0 + p * g.c0 * g.c1;
            if constexpr (VU == 2) {
                const u64x2 w = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(src));
                v[i][0] = w.x; v[i][1] = w.y;
            } else {
                v[i][0] = __builtin_nontemporal_load(src);
            }
        }
#pragma unroll
        for (int i = 0; i < NR; i++)
#pragma unroll
            for (int k = 0; k < VU; k++) tile[r0 + i * RPP][lr * VU + k] = v[i][k];
    }
    __syncthreads();
    // write: columns u (TU of them), each TP contiguous packed elements; a column takes TP/VP lanes
    constexpr int LPC = TP / VP;
    constexpr int CPP = BS / LPC;
    constexpr int NC = TU / CPP;
    {
        const int lc = t % LPC, c0 = t / LPC;
#pragma unroll
        for (int i = 0; i < NC; i++) {
            const int c = c0 + i * CPP;
            u64 *dst = packed + (u0 + c) * g.c1 * g.c2 + o * g.c2 + p0 + lc * VP;
            if constexpr (VP == 2) {
                u64x2 w;
                w.x = sw8(tile[lc * 2][c]);
                w.y = sw8(tile[lc * 2 + 1][c]);
                __builtin_nontemporal_store(w, reinterpret_cast<u64x2 *>(dst));
            } else {
                __builtin_nontemporal_store(sw8(tile[lc][c]), dst);
            }
        }
    }
}

// ablation toward the product kernel: the 64 x 64 vu1 tile with
// F & 1: XCD remap of the block index; F & 2: grid-stride loop with a
// trailing barrier; F & 4: tile decode by 64-bit runtime divisions over a
// geometry struct (as TransposeGeom)
struct G2 { long long ntu, ntp, ntiles, c1c2, c2, c0, c0c1; };
template <int F>
__global__ __launch_bounds__(256) void k_tr2(const u64 *user, u64 *packed, G2 g) {
    __shared__ u64 tile[64][65];
    const int t = threadIdx.x, lo6 = t & 63, hi2 = t >> 6;
    long long b0 = blockIdx.x;
    if (F & 1) {
        const long long nb = gridDim.x, q = nb >> 3, r = nb & 7, x = b0 & 7;
        b0 = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b0 >> 3);
    }
    for (long long b = b0; b < g.ntiles; b += gridDim.x) {
        long long tu, tp, o;
        if (F & 4) {
            long long q = b;
            tu = q % g.ntu; q /= g.ntu;
            tp = q % g.ntp; q /= g.ntp;
            o = q;
        } else {
            const unsigned q = (unsigned)b;
            tu = q % (unsigned)g.ntu;
            tp = (q / (unsigned)g.ntu) % (unsigned)g.ntp;
            o = q / (unsigned)(g.ntu * g.ntp);
        }
        const long long u0 = tu * 64, p0 = tp * 64;
        const u64 *s0 = user + u0 + lo6 + o * g.c0 + p0 * g.c0c1;
        u64 v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = __builtin_nontemporal_load(s0 + (hi2 + 4 * i) * g.c0c1);
#pragma unroll
        for (int i = 0; i < 16; i++) tile[hi2 + 4 * i][lo6] = v[i];
        __syncthreads();
        u64 *d0 = packed + u0 * g.c1c2 + o * g.c2 + p0 + lo6;
#pragma unroll
        for (int i = 0; i < 16; i++) __builtin_nontemporal_store(sw8(tile[lo6][hi2 + 4 * i]), d0 + (hi2 + 4 * i) * g.c1c2);
        if (!(F & 2)) break;
        __syncthreads();
    }
}

// the product's current shape: 64 x 64, one element per lane, plain accesses, 256 threads
__global__ __launch_bounds__(256) void k_cur(const u64 *user, u64 *packed, Geo g) {
    __shared__ u64 tile[64][65];
    const long long ntu = g.c0 / 64, ntp = g.c2 / 64;
    long long b = blockIdx.x;
    const long long tu = b % ntu; b /= ntu;
    const long long tp = b % ntp; b /= ntp;
    const long long o = b;
    const long long u0 = tu * 64, p0 = tp * 64;
    const int lo6 = threadIdx.x & 63, hi2 = threadIdx.x >> 6;
    for (int r = hi2; r < 64; r += 4) tile[r][lo6] = user[u0 + lo6 + o * g.c0 + (p0 + r) * g.c0 * g.c1];
    __syncthreads();
    for (int c = hi2; c < 64; c += 4) packed[(u0 + c) * g.c1 * g.c2 + o * g.c2 + p0 + lo6] = sw8(tile[lo6][c]);
}

__global__ void k_copy(const u64x2 *s, u64x2 *d, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { u64x2 w = __builtin_nontemporal_load(s + i); w.x = sw8(w.x); w.y = sw8(w.y); __builtin_nontemporal_store(w, d + i); }
}

struct Var { std::string name; std::function<void()> run; std::vector<float> ms; };

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 9;
    Geo g = {512, 512, 128};
    if (argc > 4) { g.c0 = atoll(argv[2]); g.c1 = atoll(argv[3]); g.c2 = atoll(argv[4]); }
    // the k_tr / k_cur variants here assume whole tiles: any other shape
    // would index past the buffers (the product kernel handles edges itself)
    if (g.c0 % 128 || g.c2 % 128 || g.c0 <= 0 || g.c1 <= 0 || g.c2 <= 0) {
        printf("C0 and C2 must be positive multiples of 128\n");
        return 2;
    }
    const long long n = g.c0 * g.c1 * g.c2;
    u64 *user, *packed, *ref;
    CK(hipMalloc(&user, n * 8));
    CK(hipMalloc(&packed, n * 8));
    CK(hipMalloc(&ref, n * 8));
    std::vector<u64> h(n);
    for (long long i = 0; i < n; i++) h[i] = (u64)i * 0x9E3779B97F4A7C15ULL;
    CK(hipMemcpy(user, h.data(), n * 8, hipMemcpyHostToDevice));
    printf("transpose %lld x %lld x %lld doubles (%.0f MiB each side), rounds %d\n", g.c0, g.c1, g.c2,
           n * 8 / 1048576.0, rounds);
    std::vector<Var> vars;
    auto add = [&](std::string nm, std::function<void()> r) { vars.push_back({nm, r, {}}); };
    add("current 64x64 v1/v1 bs256", [=] { hipLaunchKernelGGL(k_cur, dim3(n / 4096), dim3(256), 0, 0, user, ref, g); });
#define TR(TP, TU, VU, VP, BS) add(std::string("tile ") + #TP "x" #TU " vu" #VU " vp" #VP " bs" #BS, [=] { \
        hipLaunchKernelGGL((k_tr<TP, TU, VU, VP, BS>), dim3(n / (TP * TU)), dim3(BS), 0, 0, user, packed, g); });
    TR(64, 64, 1, 1, 256) TR(64, 64, 2, 2, 256)
    // longer contiguous runs per row / column (round 2)
    TR(64, 128, 1, 1, 256) TR(64, 128, 2, 1, 256) TR(64, 128, 2, 2, 256) TR(128, 64, 1, 2, 256)
    TR(128, 64, 2, 2, 256) TR(128, 128, 2, 2, 512) TR(64, 256, 2, 1, 512) TR(64, 256, 2, 2, 512)
    {
        G2 g2 = {g.c0 / 64, g.c2 / 64, n / 4096, g.c1 * g.c2, g.c2, g.c0, g.c0 * g.c1};
#define TR2(F) add(std::string("ablation flags ") + #F, [=] { hipLaunchKernelGGL((k_tr2<F>), dim3(n / 4096), dim3(256), 0, 0, user, packed, g2); });
        TR2(0) TR2(1) TR2(2) TR2(3) TR2(4) TR2(7)
    }
    {   // the product kernel (aligned path) through its own geometry
        pncxk_imap m;
        memset(&m, 0, sizeof m);
        m.ndims = 3;
        m.count[0] = g.c0; m.count[1] = g.c1; m.count[2] = g.c2;
        m.imap[0] = 1; m.imap[1] = g.c0; m.imap[2] = g.c0 * g.c1;
        m.max_count = g.c0 > g.c1 ? (g.c0 > g.c2 ? g.c0 : g.c2) : (g.c1 > g.c2 ? g.c1 : g.c2);
        pncx::TransposeGeom tg;
        if (!pncx::transpose_geom(&m, &tg)) { printf("no transpose geometry\n"); exit(1); }
        const unsigned grid = (unsigned)tg.ntiles;
        add("product k_imap_tile sc1 stores", [=] {
            hipLaunchKernelGGL((pncx::k_imap_tile<pncx::SwapOp<8>, true, true, true>), dim3(grid), dim3(256), 0, 0,
                               (const uint8_t *)user, (uint8_t *)packed, tg, 0ULL, pncx::Sink{nullptr, nullptr, 0, 0}); });
        add("product k_imap_tile (nt stores)", [=] {
            hipLaunchKernelGGL((pncx::k_imap_tile<pncx::SwapOp<8>, true, true, false>), dim3(grid), dim3(256), 0, 0,
                               (const uint8_t *)user, (uint8_t *)packed, tg, 0ULL, pncx::Sink{nullptr, nullptr, 0, 0}); });
    }
    add("flat swap copy (same bytes)", [=] { hipLaunchKernelGGL(k_copy, dim3(n / 2 / 256), dim3(256), 0, 0,
                                                                  (const u64x2 *)user, (u64x2 *)packed, n / 2); });
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto &v : vars) { v.run(); v.run(); }
    CK(hipDeviceSynchronize());
    // correctness: every tiled variant against the current kernel's output
    std::vector<u64> hr(n), hp(n);
    CK(hipMemcpy(hr.data(), ref, n * 8, hipMemcpyDeviceToHost));
    bool ok_ref = true;
    for (long long u = 0; u < g.c0 && ok_ref; u += 37)
        for (long long o = 0; o < g.c1 && ok_ref; o += 29)
            for (long long p = 0; p < g.c2; p++)
                if (hr[u * g.c1 * g.c2 + o * g.c2 + p] != __builtin_bswap64(h[u + o * g.c0 + p * g.c0 * g.c1])) { ok_ref = false; break; }
    printf("current kernel vs host transpose: %s\n", ok_ref ? "ok" : "MISMATCH");
    for (size_t k = 1; k + 1 < vars.size(); k++) {
        CK(hipMemset(packed, 0, n * 8));
        vars[k].run();
        CK(hipMemcpy(hp.data(), packed, n * 8, hipMemcpyDeviceToHost));
        if (hp != hr) printf("MISMATCH: %s\n", vars[k].name.c_str());
    }
    // each sample: one warm launch, then 10 launches of the same kernel back
    // to back between the events (round 1 timed single launches after a
    // different kernel, and the order then moved results by ~10 points:
    // the 256 MiB sides are the size of the Infinity Cache)
    for (int r = 0; r < rounds; r++)
        for (auto &v : vars) {
            v.run();
            CK(hipEventRecord(a, 0));
            for (int k = 0; k < 10; k++) v.run();
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            v.ms.push_back(ms / 10);
        }
    CK(hipGetLastError());
    const double moved = 16.0 * n;
    for (auto &v : vars) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2];
        printf("%-32s median %7.4f ms  %7.1f GB/s  (%.1f%% of 8 TB/s)\n", v.name.c_str(), med, moved / med / 1e6,
               100.0 * moved / med / 1e6 / 8000.0);
    }
    return 0;
}
