// pncx_kern.hpp -- streaming kernels of the swap / type-convert path (gfx950).
//
// One kernel template serves every conversion class.  An "Op" says how one
// source element (raw bits as loaded) becomes one destination element (raw
// bits as stored).  k_tile gives each 256-lane block one tile (a one-shot
// grid; lanes loop only past 2^23 blocks) shaped by Shape<Op>: every global
// load and store instruction of a wave covers one contiguous 1 KiB.
// The range-tested and byte-source 2:1 widening ops run two tiles per block
// (k_tile_u, Shape::TILE_U); the sign-bit byte classes convert a word at a
// time (swar_conv).
// The kernels are HBM-bound (no contraction: no MFMA).  LDS stages the
// narrow side of 4:1 / 8:1 widening and of narrowing tiles (Shape below).
//
// Status: a lane accumulates "some element was out of range"; at the end
// each wave ballots it and its first out-of-range lane stores the launch's
// epoch into the block's flag word (Sink, publish); a second kernel reduces
// the flags into the status word(s).  This is the reference's "return the
// first error" (ncx.m4:2487-2488), since NC_ERANGE is the only error a
// conversion loop can produce.
#pragma once

#include "pncx_device.hpp"
#include "pncx_shim.h"

#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

namespace pncx {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    else return *reinterpret_cast<const u32x4 *>(p);
}
// Streaming store: "nt sc1" -- nontemporal, and written through without
// keeping the line in the XCD's L2 (MI355X_MICROARCH.md: sc1 stores drop
// the line).  The 32 GiB in-place swap moved 6.82 TB/s this way against
// 6.61 TB/s with nt alone (tools/swap_sweep.hip, profiles/
// r01_swap_sweep_store_policy.txt).  No builtin exposes sc1 on a global
// store, hence the vector-store inline asm; nothing in these kernels reads
// what it stores, so the compiler's wait counting needs no view of it.
// What the compiler cannot see is the store-data hazard: on gfx940+ a VALU
// write to the VGPRs of a store with more than 64 bits of data needs 2 wait
// states (LLVM inserts them for its own stores, GCNHazardRecognizer), and a
// register reused right after this asm store corrupted the first 8 bytes of
// 16 (k_tile<PutOp<NC_FLOAT, double>>, round 2).  The s_nop 1 inside the asm
// provides them; 64-bit stores have no such hazard.
template <typename T>
__device__ __forceinline__ void st_stream(uint8_t *p, T v) {
    if constexpr (sizeof(T) == 16) {
        u32x4 w;
        __builtin_memcpy(&w, &v, 16);
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1\n\ts_nop 1" ::"v"(p), "v"(w) : "memory");
    } else if constexpr (sizeof(T) == 8) {
        uint64_t w;
        __builtin_memcpy(&w, &v, 8);
        asm volatile("global_store_dwordx2 %0, %1, off nt sc1" ::"v"(p), "v"(w) : "memory");
    } else if constexpr (sizeof(T) == 4) {
        uint32_t w;
        __builtin_memcpy(&w, &v, 4);
        asm volatile("global_store_dword %0, %1, off nt sc1" ::"v"(p), "v"(w) : "memory");
    } else if constexpr (sizeof(T) == 2) {
        uint16_t h;
        __builtin_memcpy(&h, &v, 2);
        const uint32_t w = h;
        asm volatile("global_store_short %0, %1, off nt sc1" ::"v"(p), "v"(w) : "memory");
    } else {
        // one byte per lane is half a line per wave instruction: write-through
        // of partial lines is what sc1 must not see (interleaved 16-B stores
        // fell from 55 % to 21 % of peak with sc1, tools/conv_sweep.hip), so
        // bytes keep a plain store
        static_assert(sizeof(T) == 1, "1/2/4/8/16-byte stores");
        __builtin_memcpy(p, &v, 1);
    }
}

template <bool NT>
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v) {
    if constexpr (NT) st_stream<u32x4>(p, v);
    else *reinterpret_cast<u32x4 *>(p) = v;
}

template <typename T>
__device__ __forceinline__ T ld_unaligned(const uint8_t *p) {
    T t;
    __builtin_memcpy(&t, p, sizeof t);
    return t;
}
// nontemporal load from any byte address (gfx950 global loads take
// unaligned addresses; the under-aligned type keeps the compiler honest)
template <typename T>
__device__ __forceinline__ T ld_nt_unaligned(const uint8_t *p) {
    typedef T __attribute__((aligned(1))) T1;
    return __builtin_nontemporal_load(reinterpret_cast<const T1 *>(p));
}
// nontemporal store (nt, not sc1) to any byte address
template <typename T>
__device__ __forceinline__ void st_nt_unaligned(uint8_t *p, T t) {
    typedef T __attribute__((aligned(1))) T1;
    __builtin_nontemporal_store(t, reinterpret_cast<T1 *>(p));
}
template <typename T>
__device__ __forceinline__ void st_unaligned(uint8_t *p, T t) {
    __builtin_memcpy(p, &t, sizeof t);
}

template <int A, int B> struct cmin { static constexpr int value = A < B ? A : B; };

int launch_grid(int64_t work_items, int per_thread);  // defined in pncx_kern_swap.hip

// ---------------------------------------------------------------------------
// Ops
// ---------------------------------------------------------------------------
// byte reversal of ES-byte elements (ncmpii_in_swapn / swapn?b)
template <int ES>
struct SwapOp {
    using SU = typename std::conditional<ES == 1, uint8_t,
               typename std::conditional<ES == 2, uint16_t,
               typename std::conditional<ES == 4, uint32_t, uint64_t>::type>::type>::type;
    using DU = SU;
    using fill_t = uint64_t;
    static constexpr int SS = ES, DS = ES, VEC = 16 / ES;
    static constexpr bool PRESERVE = false;
    __device__ static __forceinline__ DU one(SU s, DU, fill_t, bool &) { return bswap(s); }
};

// GET: external (big-endian raw) -> internal (native raw)
template <int XT, int IT>
struct GetOp {
    using XI = X<XT>;
    using II = I<IT>;
    using SU = typename XI::U;
    using DU = typename II::U;
    using fill_t = uint64_t;
    static constexpr int SS = XI::size, DS = II::size;
    static constexpr int VEC = 16 / cmin<SS, DS>::value;
    static constexpr bool PRESERVE = false;
    __device__ static __forceinline__ DU one(SU s, DU, fill_t, bool &bad) {
        const typename XI::T xx = bits_to<typename XI::T>(bswap(s));
        const typename II::T v = get1<XT, IT>(xx, bad);
        return bits_to<DU>(v);
    }
};

// PUT: internal (native raw) -> external (big-endian raw)
template <int XT, int IT, bool PRES>
struct PutOp {
    using XI = X<XT>;
    using II = I<IT>;
    using SU = typename II::U;
    using DU = typename XI::U;
    using fill_t = uint64_t;   // native bits of the xtype fill value
    static constexpr int SS = II::size, DS = XI::size;
    static constexpr int VEC = 16 / cmin<SS, DS>::value;
    static constexpr bool PRESERVE = PRES;
    __device__ static __forceinline__ DU one(SU s, DU old, fill_t fill, bool &bad) {
        const typename II::T v = bits_to<typename II::T>(s);
        bool b = false;
        const typename XI::T xx = put1<XT, IT>(v, bits_to<typename XI::T>((DU)fill), b);
        bad |= b;
        if constexpr (PRES) {
            // fillp == NULL: keep (1-byte) or swap (ushort/uint <- schar) the
            // bytes already in xbuf
            if (b) return bswap(old);
        }
        return bswap(bits_to<DU>(xx));
    }
};

// ---------------------------------------------------------------------------
// Word-parallel (SWAR) forms of the classes whose only range rule is the sign
// bit of a byte: per element they cost ~6 VALU (extract, compare, select,
// insert), ~100 per wave with 16 elements per lane, and ran at 72-75 % of
// peak against 83 % for the plain 1-byte copy (profiles/r03d_matrix_all.jsonl,
// r03a_pmc_pairs.txt).  Here a 32-bit word carries 4 bytes (or two 16-bit
// lanes) through masks, v_perm_b32 and packed 16-bit shifts:
//   1: schar <-> uchar (NCX_GETN_BYTE / NCX_PUTN_BYTE, ncx.m4:2369-2392,
//      2561-2581; get_NC_UBYTE_schar :2817-2834): a byte with bit 7 set is
//      out of range -> fill byte
//   2: get NC_BYTE -> ushort (NCX_GET1I, ncx.m4:560-598): negative -> 65535
//      (NC_FILL_USHORT), else zero-extended
//   3: put NC_USHORT <- schar (NCX_PUT1I, :631-665): negative -> the fill
//      value, else zero-extended, big-endian
// Results are bit-identical to Op::one element by element (the same tests).
// ---------------------------------------------------------------------------
template <int V, bool P> struct SwarK { static constexpr int value = V; static constexpr bool put = P; };
template <class Op> struct SwarKind : SwarK<0, false> {};
template <> struct SwarKind<GetOp<NC_BYTE, PNCX_ITYPE_UCHAR>> : SwarK<1, false> {};
template <> struct SwarKind<GetOp<NC_UBYTE, PNCX_ITYPE_SCHAR>> : SwarK<1, false> {};
template <> struct SwarKind<PutOp<NC_BYTE, PNCX_ITYPE_UCHAR, false>> : SwarK<1, true> {};
template <> struct SwarKind<PutOp<NC_UBYTE, PNCX_ITYPE_SCHAR, false>> : SwarK<1, true> {};
template <> struct SwarKind<GetOp<NC_BYTE, PNCX_ITYPE_USHORT>> : SwarK<2, false> {};
template <> struct SwarKind<PutOp<NC_USHORT, PNCX_ITYPE_SCHAR, false>> : SwarK<3, true> {};

typedef short s16x2 __attribute__((ext_vector_type(2)));

// 0xffff in each 16-bit lane of t whose bit 15 is set
__device__ __forceinline__ uint32_t lane16_sign_mask(uint32_t t) {
    s16x2 v;
    __builtin_memcpy(&v, &t, 4);
    v = v >> (s16x2){15, 15};          // v_pk_ashrrev_i16
    uint32_t r;
    __builtin_memcpy(&r, &v, 4);
    return r;
}

template <class Op, int K>
__device__ __forceinline__ bool swar_conv(const uint8_t *sb, uint8_t *db, uint64_t fill, bool &bad) {
    constexpr int kind = SwarKind<Op>::value;
    if constexpr (kind == 1 && K % 4 == 0) {
        constexpr int NW = K / 4;
        uint32_t fbyte;
        if constexpr (SwarKind<Op>::put) fbyte = (uint32_t)(uint8_t)fill;           // the variable's fill
        else fbyte = (uint32_t)bits_to<uint8_t>(Op::II::fill());                     // the itype default
        const uint32_t F = fbyte * 0x01010101u;
        uint32_t w[NW], acc = 0;
        __builtin_memcpy(w, sb, sizeof w);
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t m = w[k] & 0x80808080u;
            acc |= m;
            const uint32_t mm = (m << 1) - (m >> 7);       // 0xff in every byte with bit 7 set
            w[k] = (w[k] & ~mm) | (F & mm);
        }
        __builtin_memcpy(db, w, sizeof w);
        bad |= acc != 0;
        return true;
    } else if constexpr ((kind == 2 || kind == 3) && K % 4 == 0) {
        constexpr int NW = K / 4;                          // source words; two output words each
        uint32_t w[NW], o[2 * NW], acc = 0;
        __builtin_memcpy(w, sb, sizeof w);
        uint32_t F = 0;
        if constexpr (kind == 3) {
            const uint32_t f16 = (uint32_t)(uint16_t)fill;
            const uint32_t fbe = ((f16 & 0xffu) << 8) | (f16 >> 8);
            F = fbe | (fbe << 16);
        }
#pragma unroll
        for (int k = 0; k < NW; k++) {
            acc |= w[k];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                // t: byte 2h -> bits 8-15, byte 2h+1 -> bits 24-31 (the
                // big-endian ushort of a non-negative value); sign bits on top
                const uint32_t t = __builtin_amdgcn_perm(0u, w[k], h ? 0x030c020cu : 0x010c000cu);
                const uint32_t mm = lane16_sign_mask(t);
                if constexpr (kind == 2) {
                    const uint32_t e = __builtin_amdgcn_perm(0u, w[k], h ? 0x0c030c02u : 0x0c010c00u);
                    o[2 * k + h] = e | mm;                 // negative -> 0xffff
                } else {
                    o[2 * k + h] = (t & ~mm) | (F & mm);
                }
            }
        }
        __builtin_memcpy(db, o, sizeof o);
        bad |= (acc & 0x80808080u) != 0;
        return true;
    } else {
        return false;
    }
}

// ---------------------------------------------------------------------------
// Kernel: vector body over 16B-aligned [head, head + nvec*VEC) plus scalar
// head [0, head) and tail [head + nvec*VEC, n).
// ---------------------------------------------------------------------------
template <class Op>
__device__ __forceinline__ void scalar_elem(const uint8_t *src, uint8_t *dst, int64_t e,
                                            typename Op::fill_t fill, bool &bad) {
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    const SU s = ld_unaligned<SU>(src + e * Op::SS);
    DU old = 0;
    if constexpr (Op::PRESERVE) old = ld_unaligned<DU>(dst + e * Op::DS);
    st_unaligned<DU>(dst + e * Op::DS, Op::one(s, old, fill, bad));
}

template <class Op, bool NT>
__device__ __forceinline__ void vec_step(const uint8_t *src, uint8_t *dst,
                                         typename Op::fill_t fill, bool &bad) {
    constexpr int SB = Op::VEC * Op::SS, DB = Op::VEC * Op::DS;
    constexpr int NS = SB / 16, ND = DB / 16;
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    u32x4 sv[NS];
#pragma unroll
    for (int k = 0; k < NS; k++) sv[k] = ld16<NT>(src + 16 * k);
    u32x4 ov[ND];
    if constexpr (Op::PRESERVE) {
#pragma unroll
        for (int k = 0; k < ND; k++) ov[k] = ld16<false>(dst + 16 * k);
    }
    SU s[Op::VEC];
    DU d[Op::VEC];
    __builtin_memcpy(s, sv, SB);
    if constexpr (Op::PRESERVE) __builtin_memcpy(d, ov, DB);
#pragma unroll
    for (int e = 0; e < Op::VEC; e++) d[e] = Op::one(s[e], d[e], fill, bad);
    __builtin_memcpy(ov, d, DB);
#pragma unroll
    for (int k = 0; k < ND; k++) st16<NT>(dst + 16 * k, ov[k]);
}

// value: NC_ERANGE, or for batches the per-call epoch value (pncx_dev_batch
// then needs no zeroing of the status words between calls)
__device__ __forceinline__ void publish_status(int *status, bool bad, int value = NC_ERANGE) {
    if (status == nullptr) return;
    const unsigned long long m = __ballot(bad);
    // Every out-of-range wave would otherwise store into the same word: with
    // mostly-ERANGE data that serialises millions of atomics (measured 40 GB/s).
    // Read first (relaxed, agent scope: L2) and store only if not yet set.
    if (m != 0 && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1) &&
        __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != value)
        __hip_atomic_store(status, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Where a kernel reports NC_ERANGE.  With every out-of-range wave storing
// into one status word, the stores serialise at the memory side (about
// 4.5 ns each): config 4's secondary variant -- 128 x 2^20 float -> NC_SHORT,
// 18 % out of range, a fresh status value per call -- ran at 0.62 TB/s that
// way, and at 6.08 TB/s (no status at all: 6.23) when each block writes the
// call's epoch into a flag word of its own and a second kernel reduces the
// flags (tools/publish_sweep.hip V0 vs V3, profiles/r02_publish_sweep.txt).
// The launchers take a flag array per (device, stream) from sink_acquire
// (pncx_kern_swap.hip); flags == nullptr falls back to the per-wave publish.
struct Sink {
    int *status;   // status word of a single launch (k_batch: per-segment words)
    int *flags;    // per-block epoch flags of this launch, or nullptr
    int  epoch;    // this launch's flag value (never reused on one stream)
    int  sval;     // the value a status word gets
};

// fidx: the block's flag slot -- its launch index, or for the batch kernels
// the logical (XCD-remapped) block whose segment k_flags_batch looks up
__device__ __forceinline__ void publish(const Sink &s, int *status, bool bad, int64_t fidx = -1) {
    if (s.flags != nullptr) {
        // Per wave, no block barrier: the first out-of-range lane of each
        // wave stores the epoch (waves of one block store the same value
        // into the same word).  Round 2 reduced with __syncthreads_or, which
        // compiles to a three-barrier LDS reduction every wave of a block
        // waits in at its end; on a one-shot grid that tail was 2.8 LDS, ~30
        // SALU and ~25 VALU instructions per wave (profiles/r03a_pmc_pairs.txt:
        // byte -> uchar 78 % of peak against 84.6 % for byte -> schar, which
        // publishes nothing).
        const unsigned long long m = __ballot(bad);
        if (m != 0 && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)m) - 1))
            s.flags[fidx < 0 ? (int64_t)blockIdx.x : fidx] = s.epoch;
    } else {
        publish_status(status, bad, s.sval);
    }
}

// the launcher side (pncx_kern_swap.hip)
Sink sink_acquire(int *status, int sval, hipStream_t st, int64_t nblocks, bool want);
int sink_finish(const Sink &s, hipStream_t st, int64_t nblocks, int err);
int sink_finish_batch(const Sink &s, const pncxk_seg *dsegs, int nseg, int64_t nblocks, hipStream_t st, int err);

// can a conversion from S to D report NC_ERANGE at all (get1/put1 rules):
// into a floating type only double -> float is checked; from a floating type
// into an integer always; integer -> integer when D's range does not hold S's
template <class S, class D>
constexpr bool range_loss() {
    if constexpr (D::is_float) return S::is_float && S::size > D::size;
    else if constexpr (S::is_float) return true;
    else return S::lo < D::lo || S::hi > D::hi;
}
template <class Op> struct may_range { static constexpr bool value = true; };
template <int ES> struct may_range<SwapOp<ES>> { static constexpr bool value = false; };
template <int XT, int IT> struct may_range<GetOp<XT, IT>> { static constexpr bool value = range_loss<X<XT>, I<IT>>(); };
template <int XT, int IT, bool P> struct may_range<PutOp<XT, IT, P>> {
    static constexpr bool value = range_loss<I<IT>, X<XT>>();
};

// block -> segment of a batch grid: a few runs of equal sizes (e.g. NC_SHORT
// and NC_FLOAT variables; all-equal is one run) divide by a host-computed
// multiply + shift; anything else reads the device map.  One or two runs
// (every C4 batch) read the two run records with their kernel arguments and
// select; reading the whole 8-run table first cost the C4 mix kernel 3 points
// of peak against constant divisors (tools/c4_kernel_ablation.hip P1 / P6 /
// P3: 80.8 / 83.5 / 83.6 % on one pool per side).
__device__ __forceinline__ int run_segment(long long b, const pncxk_run &r) {
    return r.s0 + (int)(((unsigned long long)(b - r.b0) * r.mag) >> r.shr);
}

// ONE_FIRST: test for a single run first.  Measured both ways on the C4
// batches (tools/c4_ab.py, rotated buffer sets) with the 8-run scan: k_batch's
// float -> NC_SHORT class (one run) 1.3-2 % faster with the test, the
// same-type mix kernel (two runs) ~1 % slower, so only k_batch has it.
template <bool ONE_FIRST>
__device__ __forceinline__ int batch_segment(long long b, const int *map, const pncxk_groups &g,
                                             const pncxk_seg *segs, int nseg) {
    if (ONE_FIRST && g.n == 1) return run_segment(b, g.r[0]);
    if (g.n > 0 && g.n <= 2) {
        const bool hi = g.n == 2 && b >= g.r[1].b0;
        const long long b0 = hi ? g.r[1].b0 : g.r[0].b0;
        const unsigned long long mag = hi ? g.r[1].mag : g.r[0].mag;
        const int s0 = hi ? g.r[1].s0 : g.r[0].s0, shr = hi ? g.r[1].shr : g.r[0].shr;
        return s0 + (int)(((unsigned long long)(b - b0) * mag) >> shr);
    }
    if (g.n > 2) {
        int k = 0;
        while (k + 1 < g.n && b >= g.r[k + 1].b0) k++;
        return run_segment(b, g.r[k]);
    }
    if (map != nullptr) return map[b];
    int lo = 0, hi = nseg - 1;             // binary search (sorted by block0)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].block0 <= b) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// XCD-contiguous block order: under the observed round-robin dispatch,
// blocks b and b+8 share an XCD; remapping gives each XCD one contiguous
// address range (bijective for any nb; speed only, never correctness --
// cdna_hip_programming.md §5.5 T1 / "XCD swizzle must be bijective").
__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

// the batch kernels' logical block (segment lookup, flag slot): XCD-contiguous
// unless built with -DPNCX_BATCH_REMAP=0 (the A/B probe tools/c4_ab.py)
#ifndef PNCX_BATCH_REMAP
#define PNCX_BATCH_REMAP 1
#endif
__device__ __forceinline__ int64_t batch_block() {
    return PNCX_BATCH_REMAP ? xcd_remap(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
}

// One vector step per lane ("one-shot" grid): measured 6.6 TB/s for the
// 32 GiB in-place 8-byte swap vs <=5.5 TB/s for grid-stride loops
// (profiles/ and DESIGN.md).  For grids beyond MAX_BLOCKS the lanes loop.
constexpr int64_t MAX_BLOCKS = 1LL << 23;

template <class Op, bool NT>
__global__ __launch_bounds__(256) void k_stream(const uint8_t *src, uint8_t *dst, int64_t head,
                                                int64_t nvec, int64_t n,
                                                typename Op::fill_t fill, Sink sk) {
    constexpr int SB = Op::VEC * Op::SS, DB = Op::VEC * Op::DS;
    const int64_t nb = gridDim.x;
    const int64_t tid = xcd_remap(blockIdx.x, nb) * 256 + threadIdx.x;
    const int64_t stride = nb * 256;
    bool bad = false;

    if (blockIdx.x == 0) {  // scalar head / tail (fewer than 16 elements each)
        const int64_t tail0 = head + nvec * Op::VEC;
        if (threadIdx.x < head) scalar_elem<Op>(src, dst, threadIdx.x, fill, bad);
        if (tail0 + threadIdx.x < n) scalar_elem<Op>(src, dst, tail0 + threadIdx.x, fill, bad);
    }
    const uint8_t *vs = src + head * Op::SS;
    uint8_t *vd = dst + head * Op::DS;
    for (int64_t v = tid; v < nvec; v += stride) vec_step<Op, NT>(vs + v * SB, vd + v * DB, fill, bad);

    publish(sk, sk.status, bad);
}

// ---------------------------------------------------------------------------
// Tiled kernel (every op without the NULL-fill PRESERVE mode).  Measured on
// MI355X: with nontemporal stores, a store instruction whose 64 lanes do not
// cover one contiguous 1 KiB runs at half speed (int32->double 50% vs 83% of
// HBM peak), so every global access below is contiguous per instruction:
//   R = wide/narrow element size.
//   R <= 2 (DIRECT): a lane converts E = 16/wide elements per tile: the wide
//          side moves 16 B per lane, the narrow side 16/R B per lane.
//   R >= 4 (LDS):    the narrow side moves 16 B per lane through a 4 KiB LDS
//          tile; the wide side is R contiguous 1 KiB-per-wave instructions.
// ---------------------------------------------------------------------------
template <class Op>
struct Shape {
    static constexpr int SS = Op::SS, DS = Op::DS;
    static constexpr int W = SS > DS ? SS : DS, N = SS < DS ? SS : DS, R = W / N;
    // narrowing 2:1 also stages (16 B stores per lane instead of 8 B)
    static constexpr bool USE_LDS = R >= 4 || (R == 2 && SS > DS);
    static constexpr int LANES = 256;
    // Occupancy of the 4:1 and 8:1 tiles (either direction) is capped with
    // LDS the block does not use: the rate of a streaming tile depends on the
    // bytes the CU keeps in flight, best near 64-80 KiB.  A 256-lane 8:1
    // tile moves 36 KiB, so 2 blocks per CU; a 4:1 tile 20 KiB, 4 blocks;
    // an uncapped CU holds 8 blocks (tools/widen_sweep.hip occupancy
    // sweep, profiles/r03_occupancy_sweep_b.txt, same box: NC_BYTE ->
    // double 73.1 % at 8 blocks per CU, 79.9 % at 2; NC_SHORT -> double
    // 76.5 / 81.8 % at 8 / 4; float -> NC_BYTE 79.7 / 82.7 %; double ->
    // NC_BYTE 80.9 / 85.3 % at 8 / 2; while a 1:1 swap (8 KiB per tile)
    // falls from 84.7 % to 75.7 % at 4).  The LDS is handed out in two
    // 80 KiB halves per CU (27 KiB gave 6 blocks, 32 and 40 KiB 4, 54 and
    // 80 KiB 2), so 48 KiB gives 2 blocks per CU and 40 KiB gives 4.
    static constexpr int OCC_LDS = R >= 8 ? 48 * 1024 : R == 4 ? 40 * 1024 : 0;
    static constexpr int E = USE_LDS ? 16 / N : 16 / W;  // elements per lane per tile
    static constexpr int TILE = LANES * E;                // elements per block tile
    static constexpr int E2 = 16 / W;                     // elements per wide 16 B chunk
    static constexpr int LDS_BYTES = USE_LDS ? 16 * LANES : 16;
    // tiles per block of the direct shapes (k_tile_u): the 2:1 widening
    // tiles with a range test or from 1-byte elements keep two loads per
    // lane in flight through their conversion -- float -> (u)int64 73.0-76.3
    // -> 80.3-81.4 %, NC_BYTE -> short 78.5 -> 82.0 %, every 1:2 pair +1.2
    // to +3.5 points, short -> uint +1.7 -- while plain widening casts are
    // level or lose (NC_INT -> double, C3: 82.7 -> 82.0 % in the bench) and
    // the 1:1 tiles lose 2-10 points with two (tools/gpu_tile_u.sh,
    // profiles/r03k_matrix_u{1,2}.jsonl, profiles/r03l_c3_tile_u.txt)
    static constexpr int TILE_U = !USE_LDS && SS < DS && (SS == 1 || may_range<Op>::value) ? 2 : 1;
    // dynamic LDS requested at launch on top of the static tile
    static constexpr int PAD_LDS = OCC_LDS > LDS_BYTES ? OCC_LDS - LDS_BYTES : 0;
};

template <int B> struct VecT;
template <> struct VecT<16> { typedef uint32_t type __attribute__((ext_vector_type(4))); };
template <> struct VecT<8> { typedef uint32_t type __attribute__((ext_vector_type(2))); };
template <> struct VecT<4> { typedef uint32_t type; };
template <> struct VecT<2> { typedef uint16_t type; };
template <> struct VecT<1> { typedef uint8_t type; };

template <int B, bool NT>
__device__ __forceinline__ typename VecT<B>::type ldv(const uint8_t *p) {
    using V = typename VecT<B>::type;
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const V *>(p));
    else return *reinterpret_cast<const V *>(p);
}
template <int B, bool NT>
__device__ __forceinline__ void stv(uint8_t *p, typename VecT<B>::type v) {
    using V = typename VecT<B>::type;
    if constexpr (NT) st_stream<V>(p, v);
    else *reinterpret_cast<V *>(p) = v;
}

// convert K elements held as raw bytes (src layout) into raw bytes (dst layout)
template <class Op, int K>
__device__ __forceinline__ void conv_regs(const uint8_t *sb, uint8_t *db, typename Op::fill_t fill,
                                          bool &bad) {
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    if constexpr (SwarKind<Op>::value != 0) {
        if (swar_conv<Op, K>(sb, db, fill, bad)) return;
    }
    SU s[K];
    DU d[K];
    __builtin_memcpy(s, sb, sizeof s);
#pragma unroll
    for (int e = 0; e < K; e++) d[e] = Op::one(s[e], DU(0), fill, bad);
    __builtin_memcpy(db, d, sizeof d);
}

// one full tile: src/dst point at the tile's first element.  `lane` is the
// thread's lane in the tile's LANES; with valid == false the thread moves no
// data but still meets the tile's LDS barrier (the fused batch kernel runs
// four tiles per block, the last of which may be absent).
template <class Op, bool NT>
__device__ __forceinline__ void tile_body(const uint8_t *src, uint8_t *dst, typename Op::fill_t fill,
                                          bool &bad, uint8_t *lds, const int lane, const bool valid) {
    using S = Shape<Op>;
    constexpr int SS = S::SS, DS = S::DS, L = S::LANES;
    if constexpr (!S::USE_LDS) {
        if (!valid) return;
        constexpr int E = S::E, SB = E * SS, DB = E * DS;
        alignas(16) uint8_t sb[SB];
        alignas(16) uint8_t db[DB];
        const auto v = ldv<SB, NT>(src + lane * SB);
        __builtin_memcpy(sb, &v, SB);
        conv_regs<Op, E>(sb, db, fill, bad);
        typename VecT<DB>::type o;
        __builtin_memcpy(&o, db, DB);
        stv<DB, NT>(dst + lane * DB, o);
    } else if constexpr (SS < DS) {
        // widening: narrow src 16 B/lane -> LDS -> R wide 16 B chunks per lane
        constexpr int R = S::R, E2 = S::E2;
        using NV = typename VecT<E2 * SS>::type;
        if (valid) {
            const auto v = ldv<16, NT>(src + lane * 16);
            *reinterpret_cast<typename VecT<16>::type *>(lds + lane * 16) = v;
        }
        __syncthreads();
        if (!valid) return;
        // all R LDS reads before the first store: the streaming store is an
        // asm statement with a memory clobber, so reads after it cannot be
        // hoisted by the compiler (it issued read, wait, convert, store R
        // times in a row)
        NV w[R];
#pragma unroll
        for (int k = 0; k < R; k++) w[k] = *reinterpret_cast<const NV *>(lds + (k * L + lane) * E2 * SS);
#pragma unroll
        for (int k = 0; k < R; k++) {
            const int c = k * L + lane;                        // wide chunk index
            alignas(16) uint8_t sb[E2 * SS];
            alignas(16) uint8_t db[16];
            __builtin_memcpy(sb, &w[k], E2 * SS);
            conv_regs<Op, E2>(sb, db, fill, bad);
            typename VecT<16>::type o;
            __builtin_memcpy(&o, db, 16);
            stv<16, NT>(dst + c * 16, o);
        }
    } else {
        // narrowing: R wide 16 B chunks per lane -> LDS -> narrow 16 B/lane
        constexpr int R = S::R, E2 = S::E2;
#pragma unroll
        for (int k = 0; k < R; k++) {
            if (!valid) break;
            const int c = k * L + lane;
            alignas(16) uint8_t sb[16];
            alignas(16) uint8_t db[E2 * DS];
            const auto w = ldv<16, NT>(src + c * 16);
            __builtin_memcpy(sb, &w, 16);
            conv_regs<Op, E2>(sb, db, fill, bad);
            typename VecT<E2 * DS>::type o;
            __builtin_memcpy(&o, db, E2 * DS);
            *reinterpret_cast<typename VecT<E2 * DS>::type *>(lds + c * E2 * DS) = o;
        }
        __syncthreads();
        if (valid) stv<16, NT>(dst + lane * 16, *reinterpret_cast<const typename VecT<16>::type *>(lds + lane * 16));
    }
}

// scalar remainder [e0, n) by the L lanes of one tile
template <class Op, int L = 256>
__device__ __forceinline__ void scalar_range(const uint8_t *src, uint8_t *dst, int64_t e0, int64_t n,
                                             typename Op::fill_t fill, bool &bad, const int lane = threadIdx.x) {
    for (int64_t e = e0 + lane; e < n; e += L) scalar_elem<Op>(src, dst, e, fill, bad);
}

template <class Op, bool NT>
__global__ __launch_bounds__(Shape<Op>::LANES) void k_tile(const uint8_t *src, uint8_t *dst, int64_t head,
                                                           int64_t ntile, int64_t n, typename Op::fill_t fill,
                                                           Sink sk) {
    using S = Shape<Op>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[S::LDS_BYTES];
    bool bad = false;
    const int64_t nb = gridDim.x;
    if (blockIdx.x == 0) {                               // scalar head and remainder
        scalar_range<Op, S::LANES>(src, dst, 0, head, fill, bad);
        scalar_range<Op, S::LANES>(src, dst, head + ntile * S::TILE, n, fill, bad);
    }
    const uint8_t *ts = src + head * S::SS;
    uint8_t *td = dst + head * S::DS;
    for (int64_t t = xcd_remap(blockIdx.x, nb); t < ntile; t += nb) {
        tile_body<Op, NT>(ts + t * (int64_t)S::TILE * S::SS, td + t * (int64_t)S::TILE * S::DS, fill, bad,
                          lds, threadIdx.x, true);
        if constexpr (S::USE_LDS) __syncthreads();       // LDS reuse in the next tile
    }
    publish(sk, sk.status, bad);
}

// Direct-shape ops with U tiles per block (Shape::TILE_U): all U loads of a
// lane issued before its first convert, so a wave keeps U vectors in flight
// through a long conversion.  The loads are unpredicated (a lane past the
// last tile re-reads it), the stores predicated.
template <class Op, bool NT, int U>
__global__ __launch_bounds__(Shape<Op>::LANES) void k_tile_u(const uint8_t *src, uint8_t *dst, int64_t head,
                                                             int64_t ntile, int64_t n, typename Op::fill_t fill,
                                                             Sink sk) {
    using S = Shape<Op>;
    static_assert(!S::USE_LDS, "direct shapes only");
    constexpr int SS = S::SS, DS = S::DS, E = S::E, SB = E * SS, DB = E * DS;
    bool bad = false;
    const int64_t nb = gridDim.x;
    if (blockIdx.x == 0) {
        scalar_range<Op, S::LANES>(src, dst, 0, head, fill, bad);
        scalar_range<Op, S::LANES>(src, dst, head + ntile * S::TILE, n, fill, bad);
    }
    const uint8_t *ts = src + head * SS;
    uint8_t *td = dst + head * DS;
    const int64_t ngroup = (ntile + U - 1) / U;
    for (int64_t g = xcd_remap(blockIdx.x, nb); g < ngroup; g += nb) {
        typename VecT<SB>::type v[U];
#pragma unroll
        for (int i = 0; i < U; i++) {
            const int64_t t0 = g * U + i, t = t0 < ntile ? t0 : ntile - 1;    // unpredicated, clamped
            v[i] = ldv<SB, NT>(ts + (t * (int64_t)S::TILE + threadIdx.x * E) * SS);
        }
#pragma unroll
        for (int i = 0; i < U; i++) {
            const int64_t t = g * U + i;
            if (t < ntile) {
                alignas(16) uint8_t sb[SB];
                alignas(16) uint8_t db[DB];
                __builtin_memcpy(sb, &v[i], SB);
                conv_regs<Op, E>(sb, db, fill, bad);
                typename VecT<DB>::type o;
                __builtin_memcpy(&o, db, DB);
                stv<DB, NT>(td + (t * (int64_t)S::TILE + threadIdx.x * E) * DS, o);
            }
        }
    }
    publish(sk, sk.status, bad);
}

int tile_u(int dflt);   // PNCX_TILE_U = 1 / 2 / 4 overrides the op's TILE_U (A/B)

// fully scalar (misaligned buffers): one element per lane, byte-wise access
template <class Op>
__global__ __launch_bounds__(256) void k_scalar(const uint8_t *src, uint8_t *dst, int64_t n,
                                                typename Op::fill_t fill, Sink sk) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (int64_t e = tid; e < n; e += stride) scalar_elem<Op>(src, dst, e, fill, bad);
    publish(sk, sk.status, bad);
}

// ---------------------------------------------------------------------------
// Batched: many segments of one class in one launch.  Block b serves segment
// s with seg[s].block0 <= b < seg[s+1].block0 and handles a contiguous run of
// BATCH_STEPS vector steps of it (thread-strided inside the block, so each
// wave-instruction still moves 1 KiB contiguously).
// ---------------------------------------------------------------------------
// Block b serves tile (b - seg.block0) of the segment s with
// seg[s].block0 <= b < seg[s+1].block0 (binary search over the sorted table);
// the segment's first block also runs its scalar head and remainder.
constexpr int BATCH_STEPS = 1;  // tiles per block

// tile b of a batch class: segment lookup, the segment's scalar head and
// remainder on its first tile, the tile body, and the NC_ERANGE flag of b
template <class Op, bool NT>
__device__ __forceinline__ void batch_tile(const pncxk_seg *segs, int nseg, const int *map, const pncxk_groups &grp,
                                           const Sink &sk, long long b, bool present, int lane, uint8_t *lds) {
    using S = Shape<Op>;
    const int lo = present ? batch_segment<true>(b, map, grp, segs, nseg) : 0;
    const pncxk_seg sg = segs[lo];
    const uint8_t *src = (const uint8_t *)sg.src;
    uint8_t *dst = (uint8_t *)sg.dst;
    const typename Op::fill_t fill = sg.fill;
    const int64_t ntile = sg.nvec;     // full tiles
    bool bad = false;
    const int64_t rel = present ? b - sg.block0 : -1;
    if (rel == 0) {
        scalar_range<Op, S::LANES>(src, dst, 0, sg.head, fill, bad, lane);
        scalar_range<Op, S::LANES>(src, dst, sg.head + ntile * S::TILE, sg.n, fill, bad, lane);
    }
    tile_body<Op, NT>(src + (sg.head + rel * (int64_t)S::TILE) * S::SS,
                      dst + (sg.head + rel * (int64_t)S::TILE) * S::DS, fill, bad, lds, lane, rel >= 0 && rel < ntile);
    if (present) publish(sk, sg.status, bad, b);
}

template <class Op, bool NT>
__global__ __launch_bounds__(Shape<Op>::LANES) void k_batch(const pncxk_seg *segs, int nseg, const int *map,
                                                            pncxk_groups grp, Sink sk) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[Shape<Op>::LDS_BYTES];
    // logical block: segment lookup and flag slot
    batch_tile<Op, NT>(segs, nseg, map, grp, sk, batch_block(), true, threadIdx.x, lds);
}

// ---------------------------------------------------------------------------
// Same-type swaps of a batch (the SWAPMIX class: C4's NC_SHORT and NC_FLOAT
// iputs): a block of MIX_LANES lanes x 16 B, one nontemporal vector per
// lane, the element size read from the segment.
// ---------------------------------------------------------------------------
constexpr int MIX_LANES = PNCXK_MIX_LANES;

__device__ __forceinline__ u32x4 swap16(u32x4 v, int es) {
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
    return r;                              // es == 1: copy
}

template <int ES, int L = MIX_LANES>
__device__ __forceinline__ void mix_scalar(const uint8_t *src, uint8_t *dst, int64_t e0, int64_t e1) {
    using Op = SwapOp<ES>;
    bool bad = false;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += L) scalar_elem<Op>(src, dst, e, 0, bad);
}

// part `sub` of mix block b, run by L = MIX_LANES / parts lanes (the plan's
// block b covers MIX_LANES x 16 B; a smaller block covers a slice of it)
template <int L = MIX_LANES>
__device__ __forceinline__ void mix_block(const pncxk_seg *segs, int nseg, const int *map, const pncxk_groups &grp,
                                          long long b, int sub = 0) {
    const int s = batch_segment<false>(b, map, grp, segs, nseg);
    const pncxk_seg sg = segs[s];
    const uint8_t *src = (const uint8_t *)sg.src;
    uint8_t *dst = (uint8_t *)sg.dst;
    const int es = sg.aux;
    const int64_t rel = b - sg.block0;
    if (rel < sg.nvec) {
        const int64_t off = sg.head * es + (rel * MIX_LANES + sub * L + threadIdx.x) * 16;
        st16<true>(dst + off, swap16(ld16<true>(src + off), es));
    }
    if (rel == 0 && sub == 0) {            // scalar head and remainder (one lane per element)
        const int64_t tail0 = sg.head + sg.nvec * (int64_t)(MIX_LANES * 16 / es);
        switch (es) {
            case 1: mix_scalar<1, L>(src, dst, 0, sg.head); mix_scalar<1, L>(src, dst, tail0, sg.n); break;
            case 2: mix_scalar<2, L>(src, dst, 0, sg.head); mix_scalar<2, L>(src, dst, tail0, sg.n); break;
            case 4: mix_scalar<4, L>(src, dst, 0, sg.head); mix_scalar<4, L>(src, dst, tail0, sg.n); break;
            case 8: mix_scalar<8, L>(src, dst, 0, sg.head); mix_scalar<8, L>(src, dst, tail0, sg.n); break;
            default: break;
        }
    }
    // swaps never produce NC_ERANGE: no status
}

// One launch for a batch of two classes: a conversion class (256-lane tiles)
// and the same-type swaps (mix blocks).  Saves the second kernel's ramp and
// drain (C4's NC_ERANGE variant: float -> NC_SHORT + the NC_FLOAT swaps).
// Both classes are spread over all eight XCDs: with the conversion blocks
// first in one XCD-contiguous grid, two XCDs held 1.5x the bytes of the
// others and the launch took 0.44 ms against 0.30 ms for the two kernels
// (each XCD moves about an eighth of the chip's HBM rate).  So block b
// (round-robin dispatch: XCD x = b % 8, slot j = b / 8) takes, on every XCD,
// first its share of the conversion units, then its share of the swap units,
// each share contiguous (both unit counts padded to multiples of 8; padding
// blocks move nothing).
//   FL = 1024: a block runs four conversion tiles (one LDS barrier over 16
//              waves) or one whole mix block;
//   FL = 256:  a block runs one conversion tile, as k_batch does, or a
//              quarter of a mix block.
template <class Op, int FL>
__global__ __launch_bounds__(FL) void k_batch_fused(const pncxk_seg *asegs, int anseg, const int *amap,
                                                    pncxk_groups agrp, long long atiles, long long aunits8,
                                                    const pncxk_seg *bsegs, int bnseg, const int *bmap,
                                                    pncxk_groups bgrp, long long bblocks, long long bunits8,
                                                    Sink sk) {
    static_assert(Shape<Op>::LANES == 256 && Shape<Op>::PAD_LDS == 0, "fused: uncapped 256-lane tiles");
    constexpr int ASUB = FL / 256, BSUB = MIX_LANES / FL;
    __shared__ __attribute__((aligned(16))) uint8_t lds[ASUB * Shape<Op>::LDS_BYTES];
    const long long x = blockIdx.x & 7, j = blockIdx.x >> 3, aper = aunits8 >> 3, bper = bunits8 >> 3;
    if (j < aper) {                        // block-uniform branch: the tile barriers stay convergent
        const long long fb = x * aper + j;
        const int sub = ASUB > 1 ? threadIdx.x >> 8 : 0;
        const long long t = fb * ASUB + sub;
        batch_tile<Op, true>(asegs, anseg, amap, agrp, sk, t, t < atiles, threadIdx.x & 255,
                             lds + sub * Shape<Op>::LDS_BYTES);
    } else {
        const long long q = x * bper + (j - aper);
        if (q < bblocks * BSUB) mix_block<FL>(bsegs, bnseg, bmap, bgrp, q / BSUB, (int)(q % BSUB));
    }
}

// ---------------------------------------------------------------------------
// varm: the user buffer is laid out by imap[] (element strides per dimension,
// ncmpii_create_imaptype, create_imaptype.c:25-139).  The reference packs it
// with MPI_Pack into a contiguous cbuf and then converts (ncmpio_util.c:
// 654-689, 716-765; unpack :842-966); here the gather (put) or scatter (get)
// is fused with the conversion.  Packed element k (row-major over count[])
// lives at user element offset sum_d idx_d(k) * imap[d].
// ---------------------------------------------------------------------------
template <typename IDX>
__device__ __forceinline__ int64_t imap_offset(IDX k, const pncxk_imap &m) {
    int64_t off = 0;
#pragma unroll 1
    for (int d = m.ndims - 1; d > 0; d--) {
        const IDX c = (IDX)m.count[d];
        const IDX q = k / c;
        off += (int64_t)(k - q * c) * m.imap[d];
        k = q;
    }
    return off + (int64_t)k * m.imap[0];
}

// Derived buftype (the typemap MPI_Pack walks, dtype_decode.c:628-694 +
// ncmpio_util.c:620-652): packed element j is element r = j % tn of copy
// c = j / tn, in run b (pre[b] <= r < pre[b+1]) at byte c*extent + disp[b] +
// (r - pre[b])*ES.

// largest b in [lo, hi] with pre[b] <= r
__device__ __forceinline__ int64_t run_search(const long long *pre, int64_t r, int64_t lo, int64_t hi) {
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= r) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// tmode 7 (4-bit gap map): the gap elements before element p of a 64-element
// chunk are the sum of the chunk's nibbles 0..p (32 bytes, nibble s of byte
// s/2, low first).  Per-element decode for kernels whose lanes do not cover
// a chunk each; k_tgap scans the nibbles across the wave instead.
__device__ __forceinline__ uint32_t nib_prefix(const unsigned char *nib, int64_t q, uint32_t p) {
    const uint64_t *w = reinterpret_cast<const uint64_t *>(nib + q * 32);
    uint32_t g = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int lo = i * 16;
        uint64_t x = w[i];
        if ((int)p < lo) x = 0;
        else if ((int)p < lo + 15) x &= (1ULL << ((p - lo + 1) * 4)) - 1;
        x = (x & 0x0F0F0F0F0F0F0F0FULL) + ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL);
        g += (uint32_t)((x * 0x0101010101010101ULL) >> 56);
    }
    return g;
}

// any element (imap'ed order): uniform runs by division, tables by search
template <int ES, typename IDX>
__device__ __forceinline__ int64_t tmap_byte(int64_t j, const pncxk_imap &m) {
    const IDX c = (IDX)j / (IDX)m.tn;
    const IDX r = (IDX)j - c * (IDX)m.tn;
    if (m.tmode == 7)
        return (int64_t)c * m.textent + m.tlo + (int64_t)m.toff[r >> 6] +
               (int64_t)((r & 63) + nib_prefix(m.toff8, (int64_t)(r >> 6), (uint32_t)(r & 63))) * ES;
    if (m.tmode == 6)
        return (int64_t)c * m.textent + m.tlo + (int64_t)m.toff[r >> 6] + (int64_t)((r & 63) + m.toff8[r]) * ES;
    if (m.tmode == 5) return (int64_t)c * m.textent + m.tlo + (int64_t)m.toff[r >> 6] + m.toff16[r];
    if (m.tmode == 4) return (int64_t)c * m.textent + m.tlo + (int64_t)m.toff[r];
    if (m.tmode == 1) {
        const IDX q = r / (IDX)m.tlen;
        return (int64_t)c * m.textent + m.tdisp0 + (int64_t)q * m.tstride + (int64_t)(r - q * (IDX)m.tlen) * ES;
    }
    // the 64-element index narrows the search to the blocks of r's chunk
    const IDX q = r >> 6;
    const int64_t b = run_search(m.tpre, (int64_t)r, m.tcidx[q], m.tcidx[q + 1]);
    return (int64_t)c * m.textent + m.tdisp[b] + ((int64_t)r - m.tpre[b]) * ES;
}

// elements per lane in flight in the gather/scatter kernels (8 was slower on
// every layout: short runs 4302 -> 3222 GB/s, vector64 5369 -> 4638, round 2)
constexpr int IMAP_U = 4;

// GATHER = true: src strided (user, put); false: dst strided (user, get)
template <class Op, bool GATHER, typename IDX>
__global__ __launch_bounds__(256) void k_imap(const uint8_t *src, uint8_t *dst, int64_t n, pncxk_imap m,
                                              typename Op::fill_t fill, Sink sk) {
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    constexpr int UES = GATHER ? Op::SS : Op::DS;      // user element size
    const int64_t stride = (int64_t)gridDim.x * 256;
    bool bad = false;
    // IMAP_U elements per lane per step (a block step covers IMAP_U x 256
    // consecutive elements), all loads issued before the first store.  The
    // loads are unpredicated -- past the end a lane re-reads element n-1 --
    // since a predicated load costs a wait of its own; stores are predicated.
    for (int64_t k0 = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 * IMAP_U + threadIdx.x; k0 < n;
         k0 += stride * IMAP_U) {
        SU sv[IMAP_U];
        DU old[IMAP_U];
        int64_t uo[IMAP_U];
#pragma unroll
        for (int i = 0; i < IMAP_U; i++) {
            const int64_t k = k0 + i * 256 < n ? k0 + i * 256 : n - 1;
            const int64_t j = imap_offset<IDX>((IDX)k, m);          // user element index
            uo[i] = m.tmode ? tmap_byte<UES, IDX>(j, m) : j * UES;
            sv[i] = ld_unaligned<SU>(GATHER ? src + uo[i] : src + k * Op::SS);
            old[i] = 0;
            if constexpr (Op::PRESERVE) old[i] = ld_unaligned<DU>(GATHER ? dst + k * Op::DS : dst + uo[i]);
        }
#pragma unroll
        for (int i = 0; i < IMAP_U; i++) {
            const int64_t k = k0 + i * 256;
            // packed output (put): streaming stores, vector64 5013 -> 5355 GB/s; the
            // scattered user-side stores (get) and k_tmap_runs' run pieces keep
            // plain stores -- write-through of lines split between waves cost
            // the subarray case 24 % (5852 -> 4465 GB/s)
            if (k < n) {
                uint8_t *pd = GATHER ? dst + k * Op::DS : dst + uo[i];
                const DU o = Op::one(sv[i], old[i], fill, bad);
                if constexpr (GATHER) st_stream<DU>(pd, o);
                else st_unaligned<DU>(pd, o);
            }
        }
    }
    publish(sk, sk.status, bad);
}

// inclusive sum over the wave's 64 lanes: row shifts 1/2/4/8 inside each
// 16-lane row, then the row ends broadcast into the rows above (gfx9 DPP
// row_bcast:15 / row_bcast:31)
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);    // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);    // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);    // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);    // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Short-run tables with a gap map (tmode TM = 6: 8-bit gap counts, 7: 4-bit
// gap steps) over a contiguous count of whole copies: one wave per 64-element
// chunk of a copy, lane p = element p of the chunk.  The copy and chunk come
// from one wave-uniform division per chunk (k_imap divides every element by
// tn and decodes its imap), the chunk base is one scalar load, and the 4-bit
// map's gaps are a wave prefix sum of one nibble per lane.  IMAP_U chunks per
// wave in flight, loads before stores, unpredicated loads (lanes past the
// copy's end re-read its last element).  The map width is a template
// argument: with a run-time switch around the DPP scan the compiler dropped
// the packed index of the scan path (the store of a tmode-7 chunk went to
// c*tn + a stale register; found with an address-recording build, round 4).
template <class Op, bool GATHER, int TM>
__global__ __launch_bounds__(256) void k_tgap(const uint8_t *src, uint8_t *dst, uint32_t nunits, uint32_t nq,
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
            if constexpr (TM == 6) {
                g = m.toff8[rc];
            } else {
                static_assert(TM == 7, "k_tgap: 8-bit (6) or 4-bit (7) gap maps");
                const uint32_t b = m.toff8[(int64_t)q * 32 + (lane >> 1)];
                g = wave_inclusive_sum((b >> ((lane & 1) * 4)) & 15u);
            }
            const int64_t ub = (int64_t)c * m.textent + m.tlo + (int64_t)m.toff[q] + (int64_t)((rc & 63) + g) * UES;
            uo[i] = ub;
            // put: the user side's runs are read once -- nontemporal loads,
            // 4437 -> 4679 GB/s on the short-run layout (tools/tgap_bench.hip)
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
                // get: nt stores into the gapped user layout, 2240 -> 2622 GB/s on
                // the short-run layout (tools/tgap_bench.hip; sc1 write-through
                // is what hurt split lines in k_imap, plain nt does not)
                if constexpr (GATHER) st_stream<DU>(pd, o);
                else st_nt_unaligned<DU>(pd, o);
            }
        }
    }
    publish(sk, sk.status, bad);
}

// Uniform runs (tmode 1, the MPI vector / strided types) over a contiguous
// count, when every run holds whole 16-byte vectors: a lane moves one vector
// of E = 16 / (wider element size) elements, which never straddles a run or
// a copy, with one run division per vector instead of per element, and 16
// bytes per lane on the wider side (k_imap moves one element per lane).
// One vector per lane, one-shot grid, XCD order, as k_tile.
template <class Op, bool GATHER>
__global__ __launch_bounds__(256) void k_urun(const uint8_t *src, uint8_t *dst, int64_t nvec, pncxk_imap m,
                                              typename Op::fill_t fill, Sink sk) {
    constexpr int SS = Op::SS, DS = Op::DS, W = SS > DS ? SS : DS, E = 16 / W;
    constexpr int SB = E * SS, DB = E * DS, UES = GATHER ? SS : DS;
    bool bad = false;
    const int64_t stride = (int64_t)gridDim.x * 256;
    const uint32_t tn = (uint32_t)m.tn, tlen = (uint32_t)m.tlen;
    for (int64_t v = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x; v < nvec; v += stride) {
        const int64_t k = v * E;                              // first packed element of the vector
        const int64_t c = k / tn;
        const uint32_t r = (uint32_t)(k - c * tn), q = r / tlen, e = r - q * tlen;
        const int64_t ub = c * m.textent + m.tdisp0 + (int64_t)q * m.tstride + (int64_t)e * UES;
        const uint8_t *ps = GATHER ? src + ub : src + k * SS;
        uint8_t *pd = GATHER ? dst + k * DS : dst + ub;
        alignas(16) uint8_t sb[SB];
        alignas(16) uint8_t db[DB];
        const auto x = ldv<SB, true>(ps);
        __builtin_memcpy(sb, &x, SB);
        conv_regs<Op, E>(sb, db, fill, bad);
        typename VecT<DB>::type o;
        __builtin_memcpy(&o, db, DB);
        stv<DB, true>(pd, o);
    }
    publish(sk, sk.status, bad);
}

// varm whose fastest dimension is contiguous in the user buffer (imap 1,
// e.g. a padded array's interior) and holds whole vectors (count % V == 0,
// V = 16 / wider element size): a lane moves V elements of one row with one
// imap decode and one (possibly unaligned) 16-byte access on the wider side;
// k_imap decodes and moves one element per lane.  PNCX_IMAP_ROWS=0 (A/B).
template <class Op, bool GATHER, typename IDX>
__global__ __launch_bounds__(256) void k_imap_rows(const uint8_t *src, uint8_t *dst, int64_t nvec, pncxk_imap m,
                                                   typename Op::fill_t fill, Sink sk) {
    constexpr int SS = Op::SS, DS = Op::DS, W = SS > DS ? SS : DS, V = 16 / W;
    constexpr int UES = GATHER ? SS : DS;
    using SV = typename VecT<V * SS>::type;
    using DV = typename VecT<V * DS>::type;
    bool bad = false;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t v = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 256 + threadIdx.x; v < nvec; v += stride) {
        const int64_t k = v * V;
        const int64_t ub = imap_offset<IDX>((IDX)k, m) * UES;
        const SV x = ld_unaligned<SV>(GATHER ? src + ub : src + k * SS);
        alignas(16) uint8_t sb[V * SS];
        alignas(16) uint8_t db[V * DS];
        __builtin_memcpy(sb, &x, sizeof sb);
        conv_regs<Op, V>(sb, db, fill, bad);
        DV o;
        __builtin_memcpy(&o, db, sizeof o);
        st_unaligned<DV>(GATHER ? dst + k * DS : dst + ub, o);
    }
    publish(sk, sk.status, bad);
}

int imap_rows();      // PNCX_IMAP_ROWS (default 1)
int urun_enabled();   // PNCX_URUN (default 1)
int tmap_vec();       // PNCX_TMAP_VEC (default 1)

// Derived buftype in packed order with long runs (tmode 3, or uniform runs
// of 256..4096 elements, tmode 1): one wave per run
// piece (pieces of at most PNCX_TMAP_PIECE elements, split at commit), lanes
// along the piece -- both sides contiguous, no search.  c = copy, b = piece.
// VEC: a lane moves V = 16 / (wider element size) consecutive elements of
// the piece with one 16-byte access on the wider side (runs start at any
// element offset: unaligned vector accesses, legal on gfx950 global memory,
// as ld_unaligned already relies on); the piece's last len % V elements go
// one per lane.  PNCX_TMAP_VEC=0 moves one element per lane (A/B).
template <class Op, bool GATHER, bool VEC = false>
__global__ __launch_bounds__(256) void k_tmap_runs(const uint8_t *src, uint8_t *dst, int64_t n, pncxk_imap m,
                                                   typename Op::fill_t fill, Sink sk) {
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    constexpr int UES = GATHER ? Op::SS : Op::DS;
    constexpr int V = VEC && !Op::PRESERVE ? 16 / (Op::SS > Op::DS ? Op::SS : Op::DS) : 1;
    using SV = typename VecT<V * Op::SS>::type;
    using DV = typename VecT<V * Op::DS>::type;
    const int lane = threadIdx.x & 63;
    const int64_t total = n / m.tn * m.tnblk;            // pieces over all copies
    const int64_t nw = (int64_t)gridDim.x * 4;
    bool bad = false;
    for (int64_t g = (int64_t)xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6); g < total; g += nw) {
        const int64_t c = g / m.tnblk, b = g - c * m.tnblk;
        // uniform runs (tmode 1): run b is elements [b*tlen, (b+1)*tlen) at tdisp0 + b*tstride
        const int64_t p0 = m.tmode == 1 ? b * m.tlen : m.tpre[b];
        const int64_t len = m.tmode == 1 ? m.tlen : m.tpre[b + 1] - p0;
        const int64_t ub = c * m.textent + (m.tmode == 1 ? m.tdisp0 + b * m.tstride : m.tdisp[b]);
        const int64_t kb = c * m.tn + p0;                   // packed element of the piece
        int64_t done = 0;
        if constexpr (V > 1) {
            const int64_t ng = len / V;                     // whole vectors of the piece
            for (int64_t g0 = lane; g0 < ng; g0 += 64 * IMAP_U) {
                SV sv[IMAP_U];
#pragma unroll
                for (int i = 0; i < IMAP_U; i++) {
                    const int64_t e = (g0 + 64 * i < ng ? g0 + 64 * i : ng - 1) * V;
                    sv[i] = ld_unaligned<SV>(GATHER ? src + ub + e * UES : src + (kb + e) * Op::SS);
                }
#pragma unroll
                for (int i = 0; i < IMAP_U; i++) {
                    const int64_t e = (g0 + 64 * i) * V;
                    if (g0 + 64 * i < ng) {
                        alignas(16) uint8_t sb[V * Op::SS];
                        alignas(16) uint8_t db[V * Op::DS];
                        __builtin_memcpy(sb, &sv[i], sizeof sb);
                        conv_regs<Op, V>(sb, db, fill, bad);
                        DV o;
                        __builtin_memcpy(&o, db, sizeof o);
                        st_unaligned<DV>(GATHER ? dst + (kb + e) * Op::DS : dst + ub + e * UES, o);
                    }
                }
            }
            done = ng * V;
        }
        for (int64_t e0 = done + lane; e0 < len; e0 += 64 * IMAP_U) {     // loads first (clamped), then stores
            SU sv[IMAP_U];
            DU old[IMAP_U];
#pragma unroll
            for (int i = 0; i < IMAP_U; i++) {
                const int64_t e = e0 + 64 * i < len ? e0 + 64 * i : len - 1;
                sv[i] = ld_unaligned<SU>(GATHER ? src + ub + e * UES : src + (kb + e) * Op::SS);
                old[i] = 0;
                if constexpr (Op::PRESERVE)
                    old[i] = ld_unaligned<DU>(GATHER ? dst + (kb + e) * Op::DS : dst + ub + e * UES);
            }
#pragma unroll
            for (int i = 0; i < IMAP_U; i++) {
                const int64_t e = e0 + 64 * i;
                if (e < len)
                    st_unaligned<DU>(GATHER ? dst + (kb + e) * Op::DS : dst + ub + e * UES,
                                     Op::one(sv[i], old[i], fill, bad));
            }
        }
    }
    publish(sk, sk.status, bad);
}

// ---------------------------------------------------------------------------
// varm transpose: when the user buffer's fastest dimension U (smallest imap)
// is not the packed order's fastest dimension P (the last), per-element
// gathers touch one cache line per lane.  A tile of XT_P x XT_U elements of
// (P, U) goes through LDS instead: read coalesced along U in the user buffer,
// write coalesced along P in the packed buffer (put); the reverse for get.
// Other dimensions index the tile grid.  The conversion runs on the packed
// side.  XT_U = 128: a user row is read as one 1 KiB run (doubles) instead of
// 512 B; 64 x 128 ran at 69 % of peak against 62-64 % for 64 x 64 on the
// 512 x 512 x 128 double transpose and 72.5 against 71 % at 1024 x 1024 x 128
// (tools/transpose_sweep.hip, profiles/r02_transpose_sweep_wide_tiles.txt).
// ---------------------------------------------------------------------------
constexpr int XT_P = 64, XT_U = 128;

struct TransposeGeom {
    int64_t cp, cu;          // count[P] (merged: count[P-1] * count[P]), count[U]
    int64_t ip, iu;          // imap[P], imap[U] (user elements)
    int64_t cin, ip2;        // merged P: count[P], imap[P-1] (virtual row f = (f / cin, f % cin))
    int64_t su;              // packed stride of U
    int64_t tp, tu;          // tiles along P and U
    int64_t ntiles;          // tp * tu * outer
    int     nod;             // outer dims
    int     diag;            // skewed tile order: tile (tp, tu) runs as ((tp + diag * tu) % tp_count, tu); 0 row-major;
                             // < 0: (tp + hash(tu)) % tp_count
    int64_t ocount[PNCX_MAX_DIMS], ostride_p[PNCX_MAX_DIMS], ostride_u[PNCX_MAX_DIMS];
};

template <typename T>
__device__ __forceinline__ T ld_nt(const uint8_t *p) { return __builtin_nontemporal_load(reinterpret_cast<const T *>(p)); }
template <typename T, bool SC1 = true>
__device__ __forceinline__ void st_nt(uint8_t *p, T v) {
    if constexpr (SC1) st_stream<T>(p, v);
    else __builtin_nontemporal_store(v, reinterpret_cast<T *>(p));
}

// One tile, both buffers element-aligned.  256 threads: on the user side a
// row of XT_U elements is 128 lanes (2 rows per pass, 32 passes), on the
// packed side a column of XT_P elements is 64 lanes (4 columns per pass, 32
// passes).  All 32 loads per lane go out before anything is stored, with
// nontemporal global accesses, and per-lane addresses advance by a fixed
// row / column stride.  FULL tiles need no bounds; in a partial tile the load
// indices are clamped into the tile, so the extra lanes re-read (and
// convert) valid elements and only the stores are predicated -- a predicated
// load costs a wait of its own (5.0 -> 4.0 TB/s measured).
// user-side element offset of (virtual) tile row f: f * imap[P], or with the
// last two dimensions merged (MRG) (f / count[P]) * imap[P-1] + (f % count[P]) * imap[P]
template <bool MRG>
__device__ __forceinline__ int64_t xrow(const TransposeGeom &g, int64_t f) {
    if constexpr (MRG) {
        const uint64_t q = (uint64_t)f / (uint64_t)g.cin;
        return (int64_t)q * g.ip2 + (f - (int64_t)q * g.cin) * g.ip;
    } else {
        return f * g.ip;
    }
}

// a lane's running user-row pointer over rows f, f + RPP, f + 2 RPP, ...: with
// MRG the inner index wraps at count[P] (count[P] >= 16 > RPP: one wrap per step)
template <bool MRG, int RPP>
struct XRows {
    const uint8_t *ptr;
    int64_t p, step, wrap, cin;
    __device__ __forceinline__ XRows(const uint8_t *row0, const TransposeGeom &g, int64_t f, int64_t es) {
        ptr = row0 + xrow<MRG>(g, f) * es;
        step = RPP * g.ip * es;
        if constexpr (MRG) {
            cin = g.cin;
            p = f % g.cin;
            wrap = (g.ip2 - g.cin * g.ip) * es;
        }
    }
    __device__ __forceinline__ void next() {
        ptr += step;
        if constexpr (MRG) {
            p += RPP;
            if (p >= cin) {
                p -= cin;
                ptr += wrap;
            }
        }
    }
};

template <class Op, bool GATHER, bool FULL, typename TU, bool SC1, bool MRG = false>
__device__ __forceinline__ void xpose_tile(const uint8_t *src, uint8_t *dst, const TransposeGeom &g, int64_t pbase,
                                           int64_t ubase, int64_t p0, int64_t u0, int np, int nu,
                                           TU (*tile)[XT_U + 1], typename Op::fill_t fill, bool &bad) {
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    constexpr int UES = GATHER ? Op::SS : Op::DS;
    constexpr int PES = GATHER ? Op::DS : Op::SS;
    constexpr int RPP = 256 / XT_U, NR = XT_P / RPP;      // user side: rows per pass, passes
    constexpr int CPP = 256 / XT_P, NC = XT_U / CPP;      // packed side: columns per pass, passes
    const int lu = threadIdx.x % XT_U, ru = threadIdx.x / XT_U;     // user-side lane, row
    const int lp = threadIdx.x % XT_P, cp = threadIdx.x / XT_P;     // packed-side lane, column
    const int64_t cs = g.su * PES;                         // bytes between columns u (packed)
    if constexpr (GATHER) {
        const int cl = FULL || lu < nu ? lu : nu - 1;
        const uint8_t *s0 = src + (ubase + (u0 + cl) * g.iu) * UES;      // column cl of row 0
        TU v[NR];
        if constexpr (FULL) {
            // one running address: 32 precomputed 64-bit addresses would cost
            // 64 VGPRs on top of the 64 the data takes
            XRows<MRG, RPP> sp(s0, g, p0 + ru, UES);
#pragma unroll
            for (int i = 0; i < NR; i++, sp.next()) v[i] = ld_nt<TU>(sp.ptr);
        } else {
#pragma unroll
            for (int i = 0; i < NR; i++) {
                const int r = ru + RPP * i < np ? ru + RPP * i : np - 1;
                v[i] = ld_nt<TU>(s0 + xrow<MRG>(g, p0 + r) * UES);
            }
        }
#pragma unroll
        for (int i = 0; i < NR; i++) tile[ru + RPP * i][lu] = v[i];
        __syncthreads();
        uint8_t *d0 = dst + (pbase + u0 * g.su + p0 + lp) * PES;
        DU o[NC];
#pragma unroll
        for (int i = 0; i < NC; i++) {
            DU old = 0;
            if constexpr (Op::PRESERVE)
                if (FULL || (cp + CPP * i < nu && lp < np)) old = ld_unaligned<DU>(d0 + (cp + CPP * i) * cs);
            o[i] = Op::one(tile[lp][cp + CPP * i], old, fill, bad);
        }
        if constexpr (FULL) {
            uint8_t *dp = d0 + cp * cs;
#pragma unroll
            for (int i = 0; i < NC; i++, dp += CPP * cs) st_nt<DU, SC1>(dp, o[i]);
        } else {
#pragma unroll
            for (int i = 0; i < NC; i++)
                if (cp + CPP * i < nu && lp < np) st_nt<DU, SC1>(d0 + (cp + CPP * i) * cs, o[i]);
        }
    } else {
        const int pl = FULL || lp < np ? lp : np - 1;
        const uint8_t *s0 = src + (pbase + u0 * g.su + p0 + pl) * PES;
        SU v[NC];
        if constexpr (FULL) {
            const uint8_t *sp = s0 + cp * cs;
#pragma unroll
            for (int i = 0; i < NC; i++, sp += CPP * cs) v[i] = ld_nt<SU>(sp);
        } else {
#pragma unroll
            for (int i = 0; i < NC; i++) {
                const int c = cp + CPP * i < nu ? cp + CPP * i : nu - 1;
                v[i] = ld_nt<SU>(s0 + c * cs);
            }
        }
        // clamped duplicates convert like the element they copy: no false NC_ERANGE
#pragma unroll
        for (int i = 0; i < NC; i++) tile[lp][cp + CPP * i] = Op::one(v[i], DU(0), fill, bad);
        __syncthreads();
        uint8_t *d0 = dst + (ubase + (u0 + lu) * g.iu) * UES;             // column lu of row 0
        TU o[NR];
#pragma unroll
        for (int i = 0; i < NR; i++) o[i] = tile[ru + RPP * i][lu];
        if constexpr (FULL) {
            XRows<MRG, RPP> dp(d0, g, p0 + ru, UES);
#pragma unroll
            for (int i = 0; i < NR; i++, dp.next()) st_nt<TU, SC1>(const_cast<uint8_t *>(dp.ptr), o[i]);
        } else {
#pragma unroll
            for (int i = 0; i < NR; i++)
                if (ru + RPP * i < np && lu < nu) st_nt<TU, SC1>(d0 + xrow<MRG>(g, p0 + ru + RPP * i) * UES, o[i]);
        }
    }
}

// ALIGNED: both buffers element-aligned (checked at launch): xpose_tile.
// Otherwise the bounds-checked loops below with unaligned accesses.
// (256, 2): at least 2 waves per SIMD, i.e. two blocks per CU, which the
// 66 KiB tile allows -- unconstrained the 32 loads in flight per lane took
// 268 VGPRs and left one block per CU (56 % of peak instead of 68 %)
// SC1 = false: plain nontemporal stores -- unlike the streaming sweeps, the
// transpose runs 2 points faster without write-through (65.9 against 63.7 %
// of peak, profiles/r02_transpose_sweep_product.txt)
template <class Op, bool GATHER, bool ALIGNED, bool SC1 = false, bool MRG = false>
__global__ __launch_bounds__(256, 2) void k_imap_tile(const uint8_t *src, uint8_t *dst, TransposeGeom g,
                                                   typename Op::fill_t fill, Sink sk) {
    using SU = typename Op::SU;
    using DU = typename Op::DU;
    using TU = typename std::conditional<GATHER, SU, DU>::type;     // LDS holds user-side bits
    constexpr int UES = GATHER ? Op::SS : Op::DS;
    constexpr int PES = GATHER ? Op::DS : Op::SS;
    __shared__ TU tile[XT_P][XT_U + 1];
    const int t = threadIdx.x;
    const int lu = t % XT_U, ru = t / XT_U, lp = t % XT_P, cp = t / XT_P;
    constexpr int RPP = 256 / XT_U, CPP = 256 / XT_P;
    bool bad = false;
    const bool small = g.ntiles < (1LL << 32);          // tile decode in 32 bits (scalar divisions)
    for (int64_t b = xcd_remap(blockIdx.x, gridDim.x); b < g.ntiles; b += gridDim.x) {
        int64_t tu, tp, pbase = 0, ubase = 0;
        if (small) {
            uint32_t q = (uint32_t)b;
            tu = q % (uint32_t)g.tu;
            q /= (uint32_t)g.tu;
            tp = q % (uint32_t)g.tp;
            q /= (uint32_t)g.tp;
            for (int d = g.nod - 1; d >= 0; d--) {      // outer dims, innermost last
                const uint32_t i = q % (uint32_t)g.ocount[d];
                q /= (uint32_t)g.ocount[d];
                pbase += (int64_t)i * g.ostride_p[d];
                ubase += (int64_t)i * g.ostride_u[d];
            }
        } else {
            int64_t q = b;
            tu = q % g.tu;
            q /= g.tu;
            tp = q % g.tp;
            q /= g.tp;
            for (int d = g.nod - 1; d >= 0; d--) {
                const int64_t i = q % g.ocount[d];
                q /= g.ocount[d];
                pbase += i * g.ostride_p[d];
                ubase += i * g.ostride_u[d];
            }
        }
        // Diagonal order: neighbouring blocks (consecutive b, the ones an XCD
        // runs at the same time) take tiles of consecutive u; row-major they
        // share p0, so with a power-of-two leading dimension their packed-side
        // columns all sit at the same address bits below the 2^k stride.
        // Shifting p by u spreads them (a bijection on (tp, tu) for fixed tu).
        if (g.diag > 0) {
            tp += tu * g.diag;
            if (tp >= g.tp) tp %= g.tp;
        } else if (g.diag < 0) {
            // hashed: each u tile row starts at a pseudo-random p tile
            // (multiplicative hash of tu), still a bijection for fixed tu
            tp += (int64_t)(((uint32_t)tu * 0x9E3779B1u) >> 8) % g.tp;
            if (tp >= g.tp) tp -= g.tp;
        }
        const int64_t p0 = tp * XT_P, u0 = tu * XT_U;
        const int np = (int)(g.cp - p0 < XT_P ? g.cp - p0 : XT_P), nu = (int)(g.cu - u0 < XT_U ? g.cu - u0 : XT_U);
        if (ALIGNED) {
            if (np == XT_P && nu == XT_U)
                xpose_tile<Op, GATHER, true, TU, SC1, MRG>(src, dst, g, pbase, ubase, p0, u0, np, nu, tile, fill, bad);
            else
                xpose_tile<Op, GATHER, false, TU, SC1, MRG>(src, dst, g, pbase, ubase, p0, u0, np, nu, tile, fill, bad);
        } else if (GATHER) {
            // user -> LDS, lanes along U
            for (int r = ru; r < np; r += RPP)
                if (lu < nu)
                    tile[r][lu] = ld_unaligned<TU>(src + (ubase + (p0 + r) * g.ip + (u0 + lu) * g.iu) * UES);
            __syncthreads();
            // LDS -> convert -> packed, lanes along P
            for (int c = cp; c < nu; c += CPP)
                if (lp < np) {
                    uint8_t *pd = dst + (pbase + (u0 + c) * g.su + p0 + lp) * PES;
                    DU old = 0;
                    if constexpr (Op::PRESERVE) old = ld_unaligned<DU>(pd);
                    st_unaligned<DU>(pd, Op::one(tile[lp][c], old, fill, bad));
                }
        } else {
            // packed -> convert -> LDS, lanes along P
            for (int c = cp; c < nu; c += CPP)
                if (lp < np)
                    tile[lp][c] = Op::one(ld_unaligned<SU>(src + (pbase + (u0 + c) * g.su + p0 + lp) * PES),
                                          DU(0), fill, bad);
            __syncthreads();
            // LDS -> user, lanes along U
            for (int r = ru; r < np; r += RPP)
                if (lu < nu) st_unaligned<TU>(dst + (ubase + (p0 + r) * g.ip + (u0 + lu) * g.iu) * UES, tile[r][lu]);
        }
        __syncthreads();
    }
    publish(sk, sk.status, bad);
}

int xpose_merge();   // PNCX_XPOSE_MERGE=0 tiles P alone (A/B); default 1
int tgap_enabled();  // PNCX_TGAP=0: 8-bit gap maps (tmode 6) on k_imap
int xpose_order();   // PNCX_XPOSE_ORDER: 0 row-major tiles, 1 diagonal, k >= 2 skew k, 1000 hashed, -1 (unset) by shape

// Pick the transpose kernel for a varm layout: P = last dim, U = the other
// dim with the smallest imap; worth it when P is strided in the user buffer
// and U is (nearly) contiguous there.
// merge: when U is not P-1, tile P-1 and P as one virtual dimension of
// count[P-1] * count[P] rows.  For fixed u the packed bytes of (P-1, P) are
// one contiguous run, so 64-row tiles of it start on 512-byte boundaries of
// that run, and no cache line of the packed buffer is written by two blocks
// when the run's length is a multiple of 128 bytes.  Tiling P alone, a
// packed row of count[P] elements that is not a multiple of 128 bytes splits
// a line between neighbouring tiles at every tile edge: 1024 x 1024 x 250
// doubles (2000-byte rows) ran at 46 % of peak against 68 % for x 256, and
// x 254 at 31 % (tools/transpose_probe.py, profiles/r03n_xpose_shapes.jsonl).
inline bool transpose_geom(const pncxk_imap *m, TransposeGeom *g, bool merge) {
    const int nd = m->ndims, P = nd - 1;
    int U = -1;
    if (m->tmode != 0 || nd < 2) return false;
    for (int d = 0; d < P; d++)
        if (m->count[d] > 1 && (U < 0 || m->imap[d] < m->imap[U])) U = d;
    if (U < 0 || m->count[P] < 16 || m->count[U] < 16) return false;
    if (m->imap[P] <= 2 || m->imap[U] >= m->imap[P] || m->imap[U] > 2) return false;
    int64_t pst[PNCX_MAX_DIMS];
    int64_t s = 1;
    for (int d = nd - 1; d >= 0; d--) { pst[d] = s; s *= m->count[d]; }
    const bool mrg = merge && U < P - 1 && m->count[P - 1] > 1;
    g->cp = mrg ? m->count[P - 1] * m->count[P] : m->count[P];
    g->cu = m->count[U];
    g->ip = m->imap[P];
    g->iu = m->imap[U];
    g->cin = mrg ? m->count[P] : 0;
    g->ip2 = mrg ? m->imap[P - 1] : 0;
    g->su = pst[U];
    g->tp = (g->cp + XT_P - 1) / XT_P;
    g->tu = (g->cu + XT_U - 1) / XT_U;
    g->nod = 0;
    int64_t outer = 1;
    for (int d = 0; d < P; d++) {
        if (d == U || (mrg && d == P - 1)) continue;
        g->ocount[g->nod] = m->count[d];
        g->ostride_p[g->nod] = pst[d];
        g->ostride_u[g->nod] = m->imap[d];
        g->nod++;
        outer *= m->count[d];
    }
    g->ntiles = g->tp * g->tu * outer;
    // diagonal order for tilings of P alone: 8192 x 8192 doubles 52 -> 76 %
    // (put) and 58-61 -> 74-78 % (get), 16384 x 4096 57-59 -> 80 % (put);
    // merged 3-D shapes stay row-major: diagonal was 1-2 points slower there,
    // except x 254 (47-49 -> 50 %; profiles/r04k_xpose_order_ab.txt).
    // PNCX_XPOSE_ORDER=0 / 1 forces row-major / diagonal.
    {
        const int o = xpose_order();
        g->diag = o < 0 ? !mrg : (o == 1000 ? -1 : o);   // >= 2: skew of o tiles per u tile; 1000: hashed
    }
    return g->ntiles > 0;
}

template <class Op>
int launch_imap(const pncxk_args *a, const pncxk_imap *m, int gather) {
    if (a->n <= 0) return 0;
    const uint8_t *src = (const uint8_t *)a->src;
    uint8_t *dst = (uint8_t *)a->dst;
    const typename Op::fill_t fill = (typename Op::fill_t)a->fill;
    hipStream_t st = (hipStream_t)a->stream;
    TransposeGeom g;
    const bool want = may_range<Op>::value && a->status != nullptr;
    if constexpr (!Op::PRESERVE) {
        constexpr int W = Op::SS > Op::DS ? Op::SS : Op::DS, E = 16 / W;    // elements per vector
        const int ues = gather ? Op::SS : Op::DS, pes = gather ? Op::DS : Op::SS;
        const int64_t uvb = (int64_t)E * ues, pvb = (int64_t)E * pes;         // vector bytes, user / packed side
        const uint8_t *ubase = gather ? src : dst, *pbase = gather ? dst : src;
        if (m->tmode == 1 && m->ndims == 1 && m->imap[0] == 1 && urun_enabled() && m->tlen % E == 0 &&
            a->n % E == 0 && m->tn < (1LL << 32) && ((uintptr_t)ubase + (uintptr_t)m->tdisp0) % (uintptr_t)uvb == 0 &&
            m->tstride % uvb == 0 && m->textent % uvb == 0 && (uintptr_t)pbase % (uintptr_t)pvb == 0) {
            const int64_t nvec = a->n / E;
            const unsigned grid = (unsigned)((nvec + 255) / 256 < MAX_BLOCKS ? (nvec + 255) / 256 : MAX_BLOCKS);
            const Sink sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
            if (gather) hipLaunchKernelGGL((k_urun<Op, true>), dim3(grid), dim3(256), 0, st, src, dst, nvec, *m, fill, sk);
            else hipLaunchKernelGGL((k_urun<Op, false>), dim3(grid), dim3(256), 0, st, src, dst, nvec, *m, fill, sk);
            return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
        }
    }
    // run-major: long-run tables in packed order, and uniform runs of 256..4096
    // elements in packed order (one wave per run instead of a division per
    // element; with 64-element runs the per-wave setup made it slower:
    // vector64 5016 -> 3467 GB/s)
    if (m->tmode == 3 || (m->tmode == 1 && m->ndims == 1 && m->imap[0] == 1 && m->tlen >= 256 && m->tlen <= 4096)) {
        const int64_t pieces = a->n / m->tn * m->tnblk;
        const unsigned grid = (unsigned)((pieces + 3) / 4 < MAX_BLOCKS ? (pieces + 3) / 4 : MAX_BLOCKS);
        const Sink sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
        const bool vec = !Op::PRESERVE && tmap_vec();
        if (gather) {
            if (vec) hipLaunchKernelGGL((k_tmap_runs<Op, true, true>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
            else hipLaunchKernelGGL((k_tmap_runs<Op, true>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
        } else {
            if (vec) hipLaunchKernelGGL((k_tmap_runs<Op, false, true>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
            else hipLaunchKernelGGL((k_tmap_runs<Op, false>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
        }
        return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
    }
    const int ues = gather ? Op::SS : Op::DS, pes = gather ? Op::DS : Op::SS;
    const bool al = (uintptr_t)src % (uintptr_t)(gather ? ues : pes) == 0 &&
                    (uintptr_t)dst % (uintptr_t)(gather ? pes : ues) == 0;
    if (transpose_geom(m, &g, al && xpose_merge())) {       // the loops (unaligned) tile P alone
        // a packed U stride a little under a multiple of 2 MiB (x 254 doubles:
        // 2^21 - 2^14 B) lands the columns of concurrent tiles on few DRAM
        // channels in either tile order; skewing p0 by k tiles per u tile
        // spreads them: x 254 get 48 -> 57-59 % (k 32), put 49-51 -> 53-54 %
        // (k 8), 1024 x 260096 get 58 -> 67 %, put 53 -> 57 %
        // (profiles/r04q_xpose_skew_ab.txt).  Other strides keep the order
        // above: the skew cost 8192 x 8192 up to 36 points.
        if (xpose_order() < 0) {
            const int64_t S = g.su * pes, r = S & ((1LL << 21) - 1);
            if (r >= (1LL << 21) - (1LL << 15)) g.diag = gather ? 8 : 32;
        }
        const unsigned grid = (unsigned)(g.ntiles < MAX_BLOCKS ? g.ntiles : MAX_BLOCKS);
        const bool mrg = g.cin > 0;
        const Sink sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
        if (gather) {
            if (al && mrg) hipLaunchKernelGGL((k_imap_tile<Op, true, true, false, true>), dim3(grid), dim3(256), 0, st, src, dst, g, fill, sk);
            else if (al) hipLaunchKernelGGL((k_imap_tile<Op, true, true>), dim3(grid), dim3(256), 0, st, src, dst, g, fill, sk);
            else hipLaunchKernelGGL((k_imap_tile<Op, true, false>), dim3(grid), dim3(256), 0, st, src, dst, g, fill, sk);
        } else {
            if (al && mrg) hipLaunchKernelGGL((k_imap_tile<Op, false, true, false, true>), dim3(grid), dim3(256), 0, st, src, dst, g, fill, sk);
            else if (al) hipLaunchKernelGGL((k_imap_tile<Op, false, true>), dim3(grid), dim3(256), 0, st, src, dst, g, fill, sk);
            else hipLaunchKernelGGL((k_imap_tile<Op, false, false>), dim3(grid), dim3(256), 0, st, src, dst, g, fill, sk);
        }
        return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
    }
    const bool small = a->n < (1LL << 32) && m->max_count < (1LL << 32);
    if constexpr (!Op::PRESERVE) {
        constexpr int V = 16 / (Op::SS > Op::DS ? Op::SS : Op::DS);
        if (V > 1 && m->tmode == 0 && m->ndims > 1 && m->imap[m->ndims - 1] == 1 && m->count[m->ndims - 1] % V == 0 &&
            imap_rows()) {
            const int64_t nvec = a->n / V;
            const unsigned grid = (unsigned)((nvec + 255) / 256 < MAX_BLOCKS ? (nvec + 255) / 256 : MAX_BLOCKS);
            const Sink sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
            if (gather) {
                if (small) hipLaunchKernelGGL((k_imap_rows<Op, true, uint32_t>), dim3(grid), dim3(256), 0, st, src, dst, nvec, *m, fill, sk);
                else hipLaunchKernelGGL((k_imap_rows<Op, true, uint64_t>), dim3(grid), dim3(256), 0, st, src, dst, nvec, *m, fill, sk);
            } else {
                if (small) hipLaunchKernelGGL((k_imap_rows<Op, false, uint32_t>), dim3(grid), dim3(256), 0, st, src, dst, nvec, *m, fill, sk);
                else hipLaunchKernelGGL((k_imap_rows<Op, false, uint64_t>), dim3(grid), dim3(256), 0, st, src, dst, nvec, *m, fill, sk);
            }
            return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
        }
    }
    if ((m->tmode == 6 || m->tmode == 7) && m->ndims == 1 && m->imap[0] == 1 && m->tn > 0 && a->n % m->tn == 0 &&
        (m->tmode == 7 || tgap_enabled())) {
        const int64_t nq = (m->tn + 63) / 64, units = a->n / m->tn * nq;
        if (m->tn < (1LL << 31) && units < (1LL << 31)) {
            const int64_t blocks = (units + 4 * IMAP_U - 1) / (4 * IMAP_U);
            const unsigned grid = (unsigned)(blocks < MAX_BLOCKS ? blocks : MAX_BLOCKS);
            const Sink sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
            const uint32_t nu = (uint32_t)units, q = (uint32_t)nq;
            if (m->tmode == 7) {
                if (gather) hipLaunchKernelGGL((k_tgap<Op, true, 7>), dim3(grid), dim3(256), 0, st, src, dst, nu, q, *m, fill, sk);
                else hipLaunchKernelGGL((k_tgap<Op, false, 7>), dim3(grid), dim3(256), 0, st, src, dst, nu, q, *m, fill, sk);
            } else {
                if (gather) hipLaunchKernelGGL((k_tgap<Op, true, 6>), dim3(grid), dim3(256), 0, st, src, dst, nu, q, *m, fill, sk);
                else hipLaunchKernelGGL((k_tgap<Op, false, 6>), dim3(grid), dim3(256), 0, st, src, dst, nu, q, *m, fill, sk);
            }
            return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
        }
    }
    const int grid = launch_grid(a->n, 4);
    const Sink sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
    if (gather) {
        if (small) hipLaunchKernelGGL((k_imap<Op, true, uint32_t>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
        else hipLaunchKernelGGL((k_imap<Op, true, uint64_t>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
    } else {
        if (small) hipLaunchKernelGGL((k_imap<Op, false, uint32_t>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
        else hipLaunchKernelGGL((k_imap<Op, false, uint64_t>), dim3(grid), dim3(256), 0, st, src, dst, a->n, *m, fill, sk);
    }
    return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
}

// ---------------------------------------------------------------------------
// host-side helpers
// ---------------------------------------------------------------------------
// Elements before both pointers are aligned, to a 128-byte line when one
// head puts both there (each wave's 1 KiB then covers whole lines), else to
// the widest of 64/32/16 bytes; -1 if not even 16 bytes is reachable.
template <class Op>
inline int64_t vec_head(const void *src, const void *dst, int64_t n) {
    const uintptr_t s = (uintptr_t)src, d = (uintptr_t)dst;
    for (uintptr_t al = 128; al >= 16; al >>= 1)
        for (int64_t h = 0; h < 128 && h <= n; h++)
            if (((s + h * Op::SS) & (al - 1)) == 0 && ((d + h * Op::DS) & (al - 1)) == 0) return h;
    return -1;
}


template <class Op>
int launch_stream(const pncxk_args *a) {
    hipStream_t st = (hipStream_t)a->stream;
    const int64_t n = a->n;
    if (n <= 0) return 0;
    const int64_t h = vec_head<Op>(a->src, a->dst, n);
    const uint8_t *src = (const uint8_t *)a->src;
    uint8_t *dst = (uint8_t *)a->dst;
    const typename Op::fill_t fill = (typename Op::fill_t)a->fill;
    const bool want = may_range<Op>::value && a->status != nullptr;
    int64_t grid;
    Sink sk;
    if (h < 0) {
        grid = launch_grid(n, 1);
        sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
        hipLaunchKernelGGL((k_scalar<Op>), dim3((unsigned)grid), dim3(256), 0, st, src, dst, n, fill, sk);
    } else if constexpr (Op::PRESERVE) {
        // NULL-fill codecs read xbuf: interleaved layout, plain stores
        const int64_t nvec = (n - h) / Op::VEC;
        grid = (nvec + 255) / 256;
        if (grid < 1) grid = 1;
        if (grid > MAX_BLOCKS) grid = MAX_BLOCKS;
        sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
        hipLaunchKernelGGL((k_stream<Op, false>), dim3((unsigned)grid), dim3(256), 0, st, src, dst, h,
                           nvec, n, fill, sk);
    } else {
        const int64_t ntile = (n - h) / Shape<Op>::TILE;
        const int u = Shape<Op>::USE_LDS ? 1 : tile_u(Shape<Op>::TILE_U);
        grid = ntile < 1 ? 1 : (ntile + u - 1) / u;
        if (grid > MAX_BLOCKS) grid = MAX_BLOCKS;
        sk = sink_acquire(a->status, NC_ERANGE, st, grid, want);
        if constexpr (!Shape<Op>::USE_LDS) {
            if (u == 2 && a->nontemporal >= 0) {
                hipLaunchKernelGGL((k_tile_u<Op, true, 2>), dim3((unsigned)grid), dim3(Shape<Op>::LANES), 0, st, src,
                                   dst, h, ntile, n, fill, sk);
                return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
            }
            if (u == 4 && a->nontemporal >= 0) {
                hipLaunchKernelGGL((k_tile_u<Op, true, 4>), dim3((unsigned)grid), dim3(Shape<Op>::LANES), 0, st, src,
                                   dst, h, ntile, n, fill, sk);
                return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
            }
        }
        if (a->nontemporal >= 0)
            hipLaunchKernelGGL((k_tile<Op, true>), dim3((unsigned)grid), dim3(Shape<Op>::LANES), Shape<Op>::PAD_LDS, st,
                               src, dst, h, ntile, n, fill, sk);
        else
            hipLaunchKernelGGL((k_tile<Op, false>), dim3((unsigned)grid), dim3(Shape<Op>::LANES), Shape<Op>::PAD_LDS, st,
                               src, dst, h, ntile, n, fill, sk);
    }
    return sink_finish(sk, st, grid, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
}

template <class Op>
int launch_batch(const pncxk_batch_args *a) {
    if (a->nblocks <= 0) return 0;
    if constexpr (Op::PRESERVE) return NC_EINVAL;   // host runs these one by one
    hipStream_t st = (hipStream_t)a->stream;
    const Sink sk = sink_acquire(nullptr, a->sval, st, a->nblocks, may_range<Op>::value);
    // timing: both events are stamped by this kernel's dispatch (the flag
    // reduce is not timed)
    hipEvent_t e0 = (hipEvent_t)a->ev_start, e1 = (hipEvent_t)a->ev_stop;
    if (e0 != nullptr || e1 != nullptr)
        hipExtLaunchKernelGGL((k_batch<Op, true>), dim3((unsigned)a->nblocks), dim3(Shape<Op>::LANES),
                              Shape<Op>::PAD_LDS, st, e0, e1, 0, a->dsegs, a->nseg, a->dmap, a->grp, sk);
    else
        hipLaunchKernelGGL((k_batch<Op, true>), dim3((unsigned)a->nblocks), dim3(Shape<Op>::LANES), Shape<Op>::PAD_LDS,
                           st, a->dsegs, a->nseg, a->dmap, a->grp, sk);
    return sink_finish_batch(sk, a->dsegs, a->nseg, a->nblocks, st, hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
}

// block size of the fused batch launch: PNCX_FUSE_LANES=1024 or 256 (default)
int fuse_lanes();

template <class Op, int FL>
void launch_fused(const pncxk_batch_args *a, const pncxk_batch_args *m, const Sink &sk, hipEvent_t e0, hipEvent_t e1,
                  hipStream_t st) {
    constexpr int ASUB = FL / 256, BSUB = MIX_LANES / FL;
    const long long aunits = (a->nblocks + ASUB - 1) / ASUB;
    const long long aunits8 = (aunits + 7) & ~7LL, bunits8 = (m->nblocks * BSUB + 7) & ~7LL;
    const long long grid = aunits8 + bunits8;
    if (e0 != nullptr || e1 != nullptr)
        hipExtLaunchKernelGGL((k_batch_fused<Op, FL>), dim3((unsigned)grid), dim3(FL), 0, st, e0, e1, 0, a->dsegs,
                              a->nseg, a->dmap, a->grp, a->nblocks, aunits8, m->dsegs, m->nseg, m->dmap, m->grp,
                              m->nblocks, bunits8, sk);
    else
        hipLaunchKernelGGL((k_batch_fused<Op, FL>), dim3((unsigned)grid), dim3(FL), 0, st, a->dsegs, a->nseg, a->dmap,
                           a->grp, a->nblocks, aunits8, m->dsegs, m->nseg, m->dmap, m->grp, m->nblocks, bunits8, sk);
}

// one launch for a conversion class `a` and the same-type swap class `m`
// of one batch (k_batch_fused); PNCXK_NOFUSE when the class's tiles do not
// fit the fused block (capped occupancy, NULL-fill codecs)
template <class Op>
int launch_batch_fused(const pncxk_batch_args *a, const pncxk_batch_args *m) {
    if constexpr (Op::PRESERVE || Shape<Op>::LANES != 256 || Shape<Op>::PAD_LDS != 0) {
        return PNCXK_NOFUSE;
    } else {
        if (a->nblocks <= 0 || m->nblocks <= 0) return PNCXK_NOFUSE;
        hipStream_t st = (hipStream_t)a->stream;
        const Sink sk = sink_acquire(nullptr, a->sval, st, a->nblocks, may_range<Op>::value);
        hipEvent_t e0 = (hipEvent_t)a->ev_start, e1 = (hipEvent_t)a->ev_stop;
        if (fuse_lanes() == 1024)
            launch_fused<Op, 1024>(a, m, sk, e0, e1, st);
        else
            launch_fused<Op, 256>(a, m, sk, e0, e1, st);
        return sink_finish_batch(sk, a->dsegs, a->nseg, a->nblocks, st,
                                 hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE);
    }
}

template <class Op>
struct OpInfo {
    static void fill(pncxk_opinfo *o) {
        o->ss = Op::SS;
        o->ds = Op::DS;
        o->vec = Shape<Op>::TILE;     // elements per block tile
        o->batch_steps = BATCH_STEPS;
    }
};

}  // namespace pncx
