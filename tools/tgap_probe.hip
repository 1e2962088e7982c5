// Address check of the 4-bit gap map decode (k_tgap's wave scan) without
// dereferencing: the same unit/chunk/lane arithmetic and DPP scan as
// pncx_kern.hpp k_tgap, writing each lane's user byte offset and packed
// index to arrays that are compared on the host with the offsets the map was
// built from.  Input: tools/tgap_probe.py writes the typemap offsets.
//   hipcc --offload-arch=gfx950 -O3 -o tools/tgap_probe tools/tgap_probe.hip
//   tools/tgap_probe <offsets.bin> <copies> <textent> <esize>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
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

__global__ __launch_bounds__(256) void k_addr(const unsigned *toff, const unsigned char *nib, uint32_t nunits,
                                              uint32_t nq, uint32_t tn, int64_t textent, int es,
                                              int64_t *uo, int64_t *ko, uint32_t *gs) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t step = gridDim.x * 16;
    for (uint32_t u0 = blockIdx.x * 16; u0 < nunits; u0 += step) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            const uint32_t c = u / nq, q = u - c * nq;
            const uint32_t r = q * 64 + lane;
            const uint32_t rc = r < tn ? r : tn - 1;
            const uint32_t b = nib[(int64_t)q * 32 + (lane >> 1)];
            const uint32_t nb = (b >> ((lane & 1) * 4)) & 15u;
            const uint32_t g = wave_inclusive_sum(nb);
            if (okw) {
                const int64_t slot = (int64_t)u * 64 + lane;
                uo[slot] = (int64_t)c * textent + (int64_t)toff[q] + (int64_t)((rc & 63) + g) * es;
                ko[slot] = (int64_t)c * tn + rc;
                gs[slot] = g;
            }
        }
    }
}

int main(int argc, char **argv) {
    if (argc < 5) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<unsigned> o;
    unsigned x;
    while (fread(&x, 4, 1, f) == 1) o.push_back(x);
    fclose(f);
    const int copies = atoi(argv[2]), es = atoi(argv[4]);
    const long long textent = atoll(argv[3]);
    const uint32_t tn = (uint32_t)o.size(), nq = (tn + 63) / 64, nunits = nq * copies;
    std::vector<unsigned> base(nq);
    std::vector<unsigned char> nib(32 * (size_t)nq, 0);
    for (uint32_t e = 0; e < tn; e++) {
        if ((e & 63) == 0) { base[e >> 6] = o[e]; continue; }
        const unsigned d = (o[e] - o[e - 1]) / es - 1;
        if (o[e] <= o[e - 1] || (o[e] - o[e - 1]) % es || d > 15) { printf("map does not fit at %u\n", e); return 3; }
        nib[e >> 1] |= (unsigned char)(d << ((e & 1) * 4));
    }
    unsigned *dt; unsigned char *dn; int64_t *duo, *dko; uint32_t *dg;
    const size_t slots = (size_t)nunits * 64;
    if (hipMalloc(&dt, 4 * (size_t)nq) || hipMalloc(&dn, nib.size()) || hipMalloc(&duo, 8 * slots) ||
        hipMalloc(&dko, 8 * slots) || hipMalloc(&dg, 4 * slots)) return 4;
    hipMemcpy(dt, base.data(), 4 * (size_t)nq, hipMemcpyHostToDevice);
    hipMemcpy(dn, nib.data(), nib.size(), hipMemcpyHostToDevice);
    hipMemset(duo, 0xff, 8 * slots);
    const unsigned grid = (nunits + 15) / 16 < 4096 ? (nunits + 15) / 16 : 4096;
    hipLaunchKernelGGL(k_addr, dim3(grid), dim3(256), 0, 0, dt, dn, nunits, nq, tn, (int64_t)textent, es, duo, dko, dg);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 5; }
    std::vector<int64_t> uo(slots), ko(slots);
    std::vector<uint32_t> gs(slots);
    hipMemcpy(uo.data(), duo, 8 * slots, hipMemcpyDeviceToHost);
    hipMemcpy(ko.data(), dko, 8 * slots, hipMemcpyDeviceToHost);
    hipMemcpy(gs.data(), dg, 4 * slots, hipMemcpyDeviceToHost);
    long long bad = 0, shown = 0;
    for (uint32_t u = 0; u < nunits; u++)
        for (uint32_t l = 0; l < 64; l++) {
            const uint32_t c = u / nq, q = u % nq, r = q * 64 + l;
            if (r >= tn) continue;
            const size_t s = (size_t)u * 64 + l;
            const int64_t want = (int64_t)c * textent + o[r];
            if (uo[s] != want || ko[s] != (int64_t)c * tn + r) {
                if (shown++ < 12)
                    printf("unit %u lane %u: uo %lld want %lld (g %u) ko %lld\n", u, l, (long long)uo[s],
                           (long long)want, gs[s], (long long)ko[s]);
                bad++;
            }
        }
    printf("tn %u copies %d units %u: %lld mismatches\n", tn, copies, nunits, bad);
    return bad ? 1 : 0;
}
