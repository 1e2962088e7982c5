// Rate of the short-run gather (k_tgap's put direction, 4-bit gap-step map,
// 8-byte swap) as a standalone kernel, for A/B of its shape without
// rebuilding libpncx: U chunks per wave in flight, and plain or nontemporal
// loads of the user side.  Layout as tools/flex_bench.py short_runs: 2^23
// runs of 1..7 doubles, gaps 0..4, 8 copies (2^28 elements).
//   hipcc --offload-arch=gfx950 -O3 -o tools/tgap_bench tools/tgap_bench.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

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

template <int U, bool NTL>
float run(const uint8_t *s, uint8_t *d, uint32_t nunits, uint32_t nq, uint32_t tn, int64_t ext, const unsigned *t,
          const unsigned char *nb) {
    const unsigned grid = (nunits + 4 * U - 1) / (4 * U);
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
    for (int rep = 0; rep < 2; rep++) {
        printf("U2 %.1f  U4 %.1f  U8 %.1f  U4nt %.1f  U8nt %.1f GB/s\n",
               alg / run<2, false>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run<4, false>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run<8, false>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run<4, true>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6,
               alg / run<8, true>(s, d, nunits, nq, tn, ext, t, nbp) / 1e6);
    }
    return 0;
}
