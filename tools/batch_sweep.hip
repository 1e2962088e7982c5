// batch_sweep.hip -- standalone tuning sweep for the config-4 batch launch
// (256 iput segments, NC_SHORT 2 MiB / NC_FLOAT 4 MiB alternating, out of
// place user buffer -> xbuf).  Not part of the product; the winner is folded
// into pnetcdf_amd/csrc/pncx_kern_swap.hip.  Interleaved rounds in one
// process (cdna_hip_programming.md §5.4 rule 24).
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

struct Seg { const u32x4 *src; u32x4 *dst; long long nvec; long long block0; int esize; int pad; };
struct Groups { int n; int s0[4]; long long b0[4]; long long per[4]; };

__device__ __forceinline__ u32x4 swapv(u32x4 v, int es) {
    if (es == 4) {
        v.x = __builtin_bswap32(v.x); v.y = __builtin_bswap32(v.y);
        v.z = __builtin_bswap32(v.z); v.w = __builtin_bswap32(v.w);
    } else {  // 2-byte: swap bytes inside each 16-bit half
        v.x = ((v.x & 0x00ff00ffu) << 8) | ((v.x >> 8) & 0x00ff00ffu);
        v.y = ((v.y & 0x00ff00ffu) << 8) | ((v.y >> 8) & 0x00ff00ffu);
        v.z = ((v.z & 0x00ff00ffu) << 8) | ((v.z >> 8) & 0x00ff00ffu);
        v.w = ((v.w & 0x00ff00ffu) << 8) | ((v.w >> 8) & 0x00ff00ffu);
    }
    return v;
}

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

__device__ __forceinline__ int seg_of(long long b, const Groups &g) {
    int k = 0;
    while (k + 1 < g.n && b >= g.b0[k + 1]) k++;
    return g.s0[k] + (int)((b - g.b0[k]) / g.per[k]);
}

// K tiles of 256 x 16 B per block, all loads issued before the stores.
// REMAP: XCD-contiguous block order over the whole grid.
template <int K, int BS, bool REMAP>
__global__ __launch_bounds__(BS) void k_batch(const Seg *segs, Groups g) {
    const long long b = REMAP ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int s = seg_of(b, g);
    const Seg sg = segs[s];
    const long long rel = (b - sg.block0) * K * BS + threadIdx.x;
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_nontemporal_load(sg.src + rel + k * BS);
#pragma unroll
    for (int k = 0; k < K; k++) __builtin_nontemporal_store(swapv(v[k], sg.esize), sg.dst + rel + k * BS);
}

// reference: one contiguous out-of-place 4-byte swap of the same bytes
template <int K, int BS>
__global__ __launch_bounds__(BS) void k_flat(const u32x4 *src, u32x4 *dst, long long nvec) {
    const long long b = xcd_remap(blockIdx.x, gridDim.x);
    const long long rel = b * K * BS + threadIdx.x;
    u32x4 v[K];
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = __builtin_nontemporal_load(src + rel + k * BS);
#pragma unroll
    for (int k = 0; k < K; k++) __builtin_nontemporal_store(swapv(v[k], 4), dst + rel + k * BS);
}

// persistent: grid = CUs x occupancy, each block walks its share of tiles
template <int BS>
__global__ __launch_bounds__(BS) void k_persist(const Seg *segs, Groups g, long long ntiles) {
    for (long long b = xcd_remap(blockIdx.x, gridDim.x); b < ntiles; b += gridDim.x) {
        const int s = seg_of(b, g);
        const Seg sg = segs[s];
        const long long rel = (b - sg.block0) * BS + threadIdx.x;
        const u32x4 v = __builtin_nontemporal_load(sg.src + rel);
        __builtin_nontemporal_store(swapv(v, sg.esize), sg.dst + rel);
    }
}

struct Var {
    std::string name;
    std::function<void()> run;
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 9;
    const int nvar = 256;
    const long long nel = 1 << 20;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // one allocation per variable and side, as bench.py's C4 (torch caching allocator aside)
    std::vector<void *> bufs;
    std::vector<long long> nv(nvar);
    std::vector<int> es(nvar);
    long long total_bytes = 0;
    for (int v = 0; v < nvar; v++) {
        es[v] = v % 2 == 0 ? 2 : 4;
        nv[v] = nel * es[v] / 16;
        total_bytes += nel * es[v];
    }
    // segments sorted by size: all shorts then all floats (the host's size grouping)
    std::vector<int> order;
    for (int v = 0; v < nvar; v += 2) order.push_back(v);
    for (int v = 1; v < nvar; v += 2) order.push_back(v);
    std::vector<u32x4 *> src(nvar), dst(nvar);
    for (int v = 0; v < nvar; v++) {
        CK(hipMalloc(&src[v], nel * es[v]));
        CK(hipMalloc(&dst[v], nel * es[v]));
        CK(hipMemset(src[v], 0x5a, nel * es[v]));
    }
    u32x4 *fs, *fd;
    CK(hipMalloc(&fs, total_bytes));
    CK(hipMalloc(&fd, total_bytes));
    CK(hipMemset(fs, 0x5a, total_bytes));
    const double moved = 2.0 * total_bytes;
    printf("CUs %d, %d vars, %.0f MiB external, %.0f MiB moved, rounds %d\n", cus, nvar, total_bytes / 1048576.0,
           moved / 1048576.0, rounds);

    // device segment tables for tiles of K*BS vectors
    auto make = [&](long long tile_vec, Seg **dsegs, Groups *g, long long *nblocks) {
        std::vector<Seg> h(nvar);
        long long b = 0;
        g->n = 0;
        long long last = -1;
        for (int i = 0; i < nvar; i++) {
            const int v = order[i];
            const long long nb = nv[v] / tile_vec;
            h[i] = {src[v], dst[v], nv[v], b, es[v], 0};
            if (nb != last) { g->s0[g->n] = i; g->b0[g->n] = b; g->per[g->n] = nb; g->n++; last = nb; }
            b += nb;
        }
        CK(hipMalloc(dsegs, sizeof(Seg) * nvar));
        CK(hipMemcpy(*dsegs, h.data(), sizeof(Seg) * nvar, hipMemcpyHostToDevice));
        *nblocks = b;
    };
    // torch-like layout: one pool, src_v and dst_v adjacent in variable order
    uint8_t *pool;
    CK(hipMalloc(&pool, 2 * total_bytes));
    CK(hipMemset(pool, 0x5a, 2 * total_bytes));
    std::vector<u32x4 *> psrc(nvar), pdst(nvar);
    {
        long long off = 0;
        for (int v = 0; v < nvar; v++) {
            psrc[v] = (u32x4 *)(pool + off); off += nel * es[v];
            pdst[v] = (u32x4 *)(pool + off); off += nel * es[v];
        }
    }
    auto make_packed = [&](long long tile_vec, Seg **dsegs, Groups *g, long long *nblocks) {
        std::vector<Seg> h(nvar);
        long long b = 0;
        g->n = 0;
        long long last = -1;
        for (int i = 0; i < nvar; i++) {
            const int v = order[i];
            const long long nb = nv[v] / tile_vec;
            h[i] = {psrc[v], pdst[v], nv[v], b, es[v], 0};
            if (nb != last) { g->s0[g->n] = i; g->b0[g->n] = b; g->per[g->n] = nb; g->n++; last = nb; }
            b += nb;
        }
        CK(hipMalloc(dsegs, sizeof(Seg) * nvar));
        CK(hipMemcpy(*dsegs, h.data(), sizeof(Seg) * nvar, hipMemcpyHostToDevice));
        *nblocks = b;
    };
    std::vector<Var> vars;
    auto add = [&](std::string n, std::function<void()> r) { vars.push_back({n, r, {}}); };
#define PACKED(K, BS, RM) { Seg *d; Groups g; long long nb; make_packed((long long)(K) * (BS), &d, &g, &nb); \
      add(std::string("packed K") + #K + " bs" + #BS + " remap" + #RM, [=] { hipLaunchKernelGGL((k_batch<K, BS, RM>), dim3(nb), dim3(BS), 0, 0, d, g); }); }
#define BATCH(K, BS, RM) { Seg *d; Groups g; long long nb; make((long long)(K) * (BS), &d, &g, &nb); \
      add(std::string("batch K") + #K + " bs" + #BS + " remap" + #RM, [=] { hipLaunchKernelGGL((k_batch<K, BS, RM>), dim3(nb), dim3(BS), 0, 0, d, g); }); }
    BATCH(1, 256, false) BATCH(1, 256, true) BATCH(1, 512, false) BATCH(1, 1024, false) BATCH(1, 512, true)
    PACKED(1, 256, false) PACKED(1, 256, true) PACKED(1, 512, false) PACKED(1, 1024, false) PACKED(1, 512, true)
    PACKED(2, 256, true) PACKED(4, 256, true)
#define PERSIST(BS, OCC) { Seg *d; Groups g; long long nb; make((long long)(BS), &d, &g, &nb); \
      add(std::string("persist bs") + #BS + " x" + #OCC, [=] { hipLaunchKernelGGL((k_persist<BS>), dim3(cus * OCC), dim3(BS), 0, 0, d, g, nb); }); }
    const long long fvec = total_bytes / 16;
#define FLAT(K, BS) add(std::string("flat K") + #K + " bs" + #BS, [=] { hipLaunchKernelGGL((k_flat<K, BS>), dim3(fvec / (K * BS)), dim3(BS), 0, 0, fs, fd, fvec); });
    FLAT(1, 256) FLAT(1, 512) FLAT(1, 1024)

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
    // check the swap once (segment 1 = a float variable)
    std::vector<uint32_t> chk(16);
    CK(hipMemcpy(chk.data(), dst[1], 64, hipMemcpyDeviceToHost));
    printf("check dst[1][0] = %08x (expect 5a5a5a5a)\n", chk[0]);
    for (auto &v : vars) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
        printf("%-26s median %7.4f ms  %7.1f GB/s   best %7.1f GB/s  (%.1f%% of 8 TB/s)\n", v.name.c_str(), med,
               moved / med / 1e6, moved / mn / 1e6, 100.0 * moved / med / 1e6 / 8000.0);
    }
    return 0;
}
