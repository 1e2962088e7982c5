// tgap_runtime_switch.hip -- the round-4 k_tgap with the map width chosen at
// RUN time (m.tmode == 6 ? 8-bit counts : 4-bit steps scanned across the
// wave), as it stood in the working tree before b3832c0 made the width a
// template argument, next to the shipped compile-time kernel.  Compiled to
// gfx950 ISA only (CPU side, no GPU): tests/test_isa_tgap_switch.py reads
// the two kernels' store-address computations (VERDICT r04 "Next" 2).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S \
//         -I pnetcdf_amd/csrc -I include tools/isa/tgap_runtime_switch.hip -o -
#include "pncx_kern.hpp"

using namespace pncx;

template <class Op, bool GATHER>
__global__ __launch_bounds__(256) void k_tgap_rt(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
                                                 pncxk_imap m, typename Op::fill_t fill, Sink sk) {
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    constexpr int UES = GATHER ? Op::SS : Op::DS;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, tn = (uint32_t)m.tn;
    const uint32_t step = gridDim.x * 4 * IMAP_U;
    bool bad = false;
    for (uint32_t u0 = xcd_remap(blockIdx.x, gridDim.x) * 4 * IMAP_U; u0 < nunits; u0 += step) {
        SU sv[IMAP_U];
        DU old[IMAP_U];
        int64_t uo[IMAP_U], ko[IMAP_U];
        bool ok[IMAP_U];
#pragma unroll
        for (int i = 0; i < IMAP_U; i++) {
            uint32_t u = u0 + i * 4 + w;
            const bool okw = u < nunits;
            u = __builtin_amdgcn_readfirstlane(okw ? u : nunits - 1);
            const uint32_t c = u / nq, q = u - c * nq;
            const uint32_t r = q * 64 + lane;
            const uint32_t rc = r < tn ? r : tn - 1;
            ok[i] = okw && r < tn;
            ko[i] = (int64_t)c * tn + rc;
            uint32_t g;
            if (m.tmode == 6) {                       /* the run-time switch */
                g = m.toff8[rc];
            } else {
                const uint32_t b = m.toff8[(int64_t)q * 32 + (lane >> 1)];
                g = wave_inclusive_sum((b >> ((lane & 1) * 4)) & 15u);
            }
            const int64_t ub = (int64_t)c * m.textent + m.tlo + (int64_t)m.toff[q] + (int64_t)((rc & 63) + g) * UES;
            uo[i] = ub;
            if constexpr (GATHER) sv[i] = ld_nt_unaligned<SU>(src + uo[i]);
            else sv[i] = ld_unaligned<SU>(src + ko[i] * Op::SS);
            old[i] = 0;
            if constexpr (Op::PRESERVE) old[i] = ld_unaligned<DU>(GATHER ? dst + ko[i] * Op::DS : dst + uo[i]);
        }
#pragma unroll
        for (int i = 0; i < IMAP_U; i++) {
            if (ok[i]) {
                uint8_t *pd = GATHER ? dst + ko[i] * Op::DS : dst + uo[i];
                const DU o = Op::one(sv[i], old[i], fill, bad);
                if constexpr (GATHER) st_stream<DU>(pd, o);
                else st_nt_unaligned<DU>(pd, o);
            }
        }
    }
    publish(sk, sk.status, bad);
}

// the faulting instance (tests/test_gpu_flex.py::test_flex_large_table:
// NC_INT written from double through a short-run typemap) and the shipped one
using FaultOp = PutOp<NC_INT, PNCX_ITYPE_DOUBLE, false>;
template __global__ void k_tgap_rt<FaultOp, true>(const uint8_t *, uint8_t *, uint32_t, uint32_t, pncxk_imap,
                                                  FaultOp::fill_t, Sink);
namespace pncx {
template __global__ void k_tgap<FaultOp, true, 7>(const uint8_t *, uint8_t *, uint32_t, uint32_t, pncxk_imap,
                                                  FaultOp::fill_t, Sink);
}
