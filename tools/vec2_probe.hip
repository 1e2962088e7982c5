// vec2_probe.hip -- the put (gather) of an MPI vector buftype with one
// element per block (MPI_Type_vector(n, 1, s, MPI_DOUBLE), s = 2 or 4) into a
// packed NC_DOUBLE buffer, with the 8-byte swap: how many packed elements a
// lane should own and how wide its user-side loads should be.  Not product
// code; the product runs this layout through k_imap (tmode 1, four elements
// per lane a grid stride apart).  Round-5 result: the shape of
// gs4 is the best with the decode in it, and a product kernel of that shape
// ran level with k_imap (profiles/r05i_vector_ab.txt), so none was kept.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/vec2_probe tools/vec2_probe.hip
//   tools/vec2_probe [stride]          rates in GB/s of algorithmic bytes (16 per element)
//
// Variants (n = 2^28 packed elements, one-shot grids, XCD order as k_tile):
//   e1     one element per lane: an 8-byte load at j*s*8, an 8-byte store (k_imap's shape)
//   e2     two consecutive packed elements per lane: two 8-byte loads, one 16-byte store
//   e4     four per lane: four 8-byte loads, two 16-byte stores
//   w2     two per lane, 16-byte loads of (element, gap) pairs, the low halves stored (s = 2)
//   copy   the contiguous control: 16 bytes in, 16 bytes out per lane (no gaps)
//   e1div  e1 with the uniform-run decode (two 32-bit divisions by run-time values)
//   gs4    four elements per lane a grid stride apart, decode as e1div (k_imap's shape)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(2); } } while (0)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
    // blocks b, b+8, b+16, ... run on one XCD: give each XCD a contiguous range
    const uint32_t per = nb / 8, rem = nb % 8, x = b % 8, k = b / 8;
    return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + k;
}

template <int V>
__global__ __launch_bounds__(256) void k_elems(const uint8_t *u, uint8_t *x, int64_t n, int s) {
    const int64_t j0 = ((int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x) * V;
    if (j0 >= n) return;
    uint64_t v[V];
#pragma unroll
    for (int k = 0; k < V; k++)
        v[k] = __builtin_nontemporal_load((const uint64_t *)(u + (j0 + k) * s * 8));
    if constexpr (V == 1) {
        __builtin_nontemporal_store(__builtin_bswap64(v[0]), (uint64_t *)(x + j0 * 8));
    } else {
#pragma unroll
        for (int k = 0; k < V; k += 2) {
            u64x2 w = {__builtin_bswap64(v[k]), __builtin_bswap64(v[k + 1])};
            __builtin_nontemporal_store(w, (u64x2 *)(x + (j0 + k) * 8));
        }
    }
}

// e1 with the generic uniform-run index math of a committed MPI vector type:
// copy c = j / tn, block q = r / tlen, element e = r % tlen (32-bit divisions
// by run-time values), as a product kernel would do it
__global__ __launch_bounds__(256) void k_e1div(const uint8_t *u, uint8_t *x, int64_t n, uint32_t tn, uint32_t tlen,
                                               int64_t tstride, int64_t textent, int64_t tdisp0) {
    const int64_t j = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x;
    if (j >= n) return;
    const uint32_t c = (uint32_t)j / tn, r = (uint32_t)j - c * tn, q = r / tlen, e = r - q * tlen;
    const int64_t ub = (int64_t)c * textent + tdisp0 + (int64_t)q * tstride + (int64_t)e * 8;
    const uint64_t v = __builtin_nontemporal_load((const uint64_t *)(u + ub));
    __builtin_nontemporal_store(__builtin_bswap64(v), (uint64_t *)(x + j * 8));
}

// grid-stride with 4 loads per lane in flight (k_imap's shape, index math as e1div)
__global__ __launch_bounds__(256) void k_gs4(const uint8_t *u, uint8_t *x, int64_t n, uint32_t tn, uint32_t tlen,
                                             int64_t tstride, int64_t textent, int64_t tdisp0) {
    const int64_t step = (int64_t)gridDim.x * 256;
    for (int64_t j0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x; j0 < n; j0 += 4 * step) {
        uint64_t v[4];
        int64_t jj[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            int64_t j = j0 + k * step;
            jj[k] = j;
            if (j >= n) j = n - 1;
            const uint32_t c = (uint32_t)j / tn, r = (uint32_t)j - c * tn, q = r / tlen, e = r - q * tlen;
            const int64_t ub = (int64_t)c * textent + tdisp0 + (int64_t)q * tstride + (int64_t)e * 8;
            v[k] = __builtin_nontemporal_load((const uint64_t *)(u + ub));
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (jj[k] < n) __builtin_nontemporal_store(__builtin_bswap64(v[k]), (uint64_t *)(x + jj[k] * 8));
    }
}

__global__ __launch_bounds__(256) void k_wide2(const uint8_t *u, uint8_t *x, int64_t n) {
    const int64_t j0 = ((int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x) * 2;
    if (j0 >= n) return;
    const u64x2 a = __builtin_nontemporal_load((const u64x2 *)(u + j0 * 16));
    const u64x2 b = __builtin_nontemporal_load((const u64x2 *)(u + (j0 + 1) * 16));
    u64x2 w = {__builtin_bswap64(a.x), __builtin_bswap64(b.x)};
    __builtin_nontemporal_store(w, (u64x2 *)(x + j0 * 8));
}

__global__ __launch_bounds__(256) void k_copy(const uint8_t *u, uint8_t *x, int64_t n) {
    const int64_t j0 = ((int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x) * 2;
    if (j0 >= n) return;
    const u64x2 a = __builtin_nontemporal_load((const u64x2 *)(u + j0 * 8));
    u64x2 w = {__builtin_bswap64(a.x), __builtin_bswap64(a.y)};
    __builtin_nontemporal_store(w, (u64x2 *)(x + j0 * 8));
}

template <class F>
static float timeit(F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipEventRecord(a, 0));
    for (int k = 0; k < 10; k++) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / 10;
}

int main(int argc, char **argv) {
    const int s = argc > 1 ? atoi(argv[1]) : 2;
    const int64_t n = 1LL << 28;
    uint8_t *u, *x;
    CK(hipMalloc(&u, (size_t)n * s * 8));
    CK(hipMalloc(&x, (size_t)n * 8));
    CK(hipMemset(u, 7, (size_t)n * s * 8));
    const double alg = (double)n * 16;
    auto grid = [&](int per) { return (unsigned)((n / per + 255) / 256); };
    // correctness: e1, e2, e4 (and w2 at s = 2) give the same packed bytes
    {
        std::vector<uint64_t> h((size_t)n * s);
        for (size_t i = 0; i < h.size(); i++) h[i] = i * 0x9E3779B97F4A7C15ULL;
        CK(hipMemcpy(u, h.data(), h.size() * 8, hipMemcpyHostToDevice));
        std::vector<uint64_t> r0(n), r1(n);
        hipLaunchKernelGGL(k_elems<1>, dim3(grid(1)), dim3(256), 0, 0, u, x, n, s);
        CK(hipMemcpy(r0.data(), x, n * 8, hipMemcpyDeviceToHost));
        bool ok = true;
        for (int64_t j = 0; j < n && ok; j += 4099) ok = r0[j] == __builtin_bswap64(h[j * s]);
        printf("# e1 %s\n", ok ? "correct" : "WRONG");
        for (int m = 0; m < 3; m++) {
            if (m == 2 && s != 2) continue;
            CK(hipMemset(x, 0, n * 8));
            if (m == 0) hipLaunchKernelGGL(k_elems<2>, dim3(grid(2)), dim3(256), 0, 0, u, x, n, s);
            if (m == 1) hipLaunchKernelGGL(k_elems<4>, dim3(grid(4)), dim3(256), 0, 0, u, x, n, s);
            if (m == 2) hipLaunchKernelGGL(k_wide2, dim3(grid(2)), dim3(256), 0, 0, u, x, n);
            CK(hipMemcpy(r1.data(), x, n * 8, hipMemcpyDeviceToHost));
            printf("# %s %s e1\n", m == 0 ? "e2" : m == 1 ? "e4" : "w2", r0 == r1 ? "matches" : "DIFFERS from");
        }
    }
    for (int rep = 0; rep < 3; rep++) {
        const float t1 = timeit([&] { hipLaunchKernelGGL(k_elems<1>, dim3(grid(1)), dim3(256), 0, 0, u, x, n, s); });
        const float t2 = timeit([&] { hipLaunchKernelGGL(k_elems<2>, dim3(grid(2)), dim3(256), 0, 0, u, x, n, s); });
        const float t4 = timeit([&] { hipLaunchKernelGGL(k_elems<4>, dim3(grid(4)), dim3(256), 0, 0, u, x, n, s); });
        const float tw = s == 2 ? timeit([&] { hipLaunchKernelGGL(k_wide2, dim3(grid(2)), dim3(256), 0, 0, u, x, n); }) : 0;
        const float tc = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(grid(2)), dim3(256), 0, 0, u, x, n); });
        const float td = timeit([&] { hipLaunchKernelGGL(k_e1div, dim3(grid(1)), dim3(256), 0, 0, u, x, n, (uint32_t)n, 1u,
                                                         (int64_t)s * 8, (int64_t)n * s * 8, (int64_t)0); });
        const unsigned gg = (unsigned)(((n + 3) / 4 + 255) / 256 < 1024 * 256 ? ((n + 3) / 4 + 255) / 256 : 1024 * 256);
        const float tg = timeit([&] { hipLaunchKernelGGL(k_gs4, dim3(gg), dim3(256), 0, 0, u, x, n, (uint32_t)n, 1u,
                                                         (int64_t)s * 8, (int64_t)n * s * 8, (int64_t)0); });
        printf("stride %d: e1 %.1f  e1div %.1f  gs4 %.1f  e2 %.1f  e4 %.1f  w2 %.1f  copy %.1f GB/s (algorithmic; the gather reads %d x the bytes)\n",
               s, alg / t1 / 1e6, alg / td / 1e6, alg / tg / 1e6, alg / t2 / 1e6, alg / t4 / 1e6, tw > 0 ? alg / tw / 1e6 : 0.0,
               alg / tc / 1e6, s);
    }
    return 0;
}
