// pncx_device.hpp -- device-side element semantics of the XDR swap / NC type
// conversion path, written for gfx950 (CDNA4).
//
// One function per direction (get1: external -> internal, put1: internal ->
// external), specialised at compile time on (xtype, itype).  The rules are
// those of PnetCDF's ncx.m4 with ERANGE_FILL (macros cited per rule below);
// the float->int casts reproduce what the reference's
// x86-64 gcc -O2 build does for NaN and for the 2^63 / 2^64 edges, because
// the GPU conversion instructions differ there (v_cvt_i32_f64(NaN) = 0).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "../../include/pncx.h"

namespace pncx {

// ---------------------------------------------------------------------------
// external types (pnetcdf.h.in:66-83) and their limits (ncx_h.m4:81-106)
// ---------------------------------------------------------------------------
template <int XT> struct X;
#define PNCX_XDEF(XT_, CT_, UT_, FLT_, LO_, HI_, FILL_)                     \
    template <> struct X<XT_> {                                           \
        using T = CT_;                                                    \
        using U = UT_;                                                    \
        static constexpr int size = sizeof(CT_);                          \
        static constexpr bool is_float = FLT_;                            \
        static constexpr long long lo = LO_;                              \
        static constexpr unsigned long long hi = HI_;                     \
        __device__ static constexpr T fill() { return (T)(FILL_); }       \
    };
PNCX_XDEF(NC_BYTE,   int8_t,   uint8_t,  false, -128, 127ull, -127)
PNCX_XDEF(NC_UBYTE,  uint8_t,  uint8_t,  false, 0, 255ull, 255)
PNCX_XDEF(NC_SHORT,  int16_t,  uint16_t, false, -32768, 32767ull, -32767)
PNCX_XDEF(NC_USHORT, uint16_t, uint16_t, false, 0, 65535ull, 65535)
PNCX_XDEF(NC_INT,    int32_t,  uint32_t, false, -2147483647LL - 1, 2147483647ull, -2147483647)
PNCX_XDEF(NC_UINT,   uint32_t, uint32_t, false, 0, 4294967295ull, 4294967295u)
PNCX_XDEF(NC_FLOAT,  float,    uint32_t, true, 0, 0, 9.9692099683868690e+36f)
PNCX_XDEF(NC_DOUBLE, double,   uint64_t, true, 0, 0, 9.9692099683868690e+36)
PNCX_XDEF(NC_INT64,  int64_t,  uint64_t, false, -9223372036854775807LL - 1, 9223372036854775807ull,
          -9223372036854775806LL)
PNCX_XDEF(NC_UINT64, uint64_t, uint64_t, false, 0, 18446744073709551615ull, 18446744073709551614ull)
#undef PNCX_XDEF

// ---------------------------------------------------------------------------
// internal types (convert_swap.m4:218-245) with their get-side default fill
// (FillDefaultValue, ncx.m4:97-111: long -> NC_FILL_INT)
// ---------------------------------------------------------------------------
template <int IT> struct I;
#define PNCX_IDEF(IT_, CT_, UT_, FLT_, LO_, HI_, FILL_)                     \
    template <> struct I<IT_> {                                           \
        using T = CT_;                                                    \
        using U = UT_;                                                    \
        static constexpr int size = sizeof(CT_);                          \
        static constexpr bool is_float = FLT_;                            \
        static constexpr long long lo = LO_;                              \
        static constexpr unsigned long long hi = HI_;                     \
        __device__ static constexpr T fill() { return (T)(FILL_); }       \
    };
PNCX_IDEF(PNCX_ITYPE_SCHAR,     int8_t,   uint8_t,  false, -128, 127ull, -127)
PNCX_IDEF(PNCX_ITYPE_UCHAR,     uint8_t,  uint8_t,  false, 0, 255ull, 255)
PNCX_IDEF(PNCX_ITYPE_SHORT,     int16_t,  uint16_t, false, -32768, 32767ull, -32767)
PNCX_IDEF(PNCX_ITYPE_USHORT,    uint16_t, uint16_t, false, 0, 65535ull, 65535)
PNCX_IDEF(PNCX_ITYPE_INT,       int32_t,  uint32_t, false, -2147483647LL - 1, 2147483647ull, -2147483647)
PNCX_IDEF(PNCX_ITYPE_UINT,      uint32_t, uint32_t, false, 0, 4294967295ull, 4294967295u)
PNCX_IDEF(PNCX_ITYPE_LONG,      int64_t,  uint64_t, false, -9223372036854775807LL - 1,
          9223372036854775807ull, -2147483647)
PNCX_IDEF(PNCX_ITYPE_FLOAT,     float,    uint32_t, true, 0, 0, 9.9692099683868690e+36f)
PNCX_IDEF(PNCX_ITYPE_DOUBLE,    double,   uint64_t, true, 0, 0, 9.9692099683868690e+36)
PNCX_IDEF(PNCX_ITYPE_LONGLONG,  int64_t,  uint64_t, false, -9223372036854775807LL - 1,
          9223372036854775807ull, -9223372036854775806LL)
PNCX_IDEF(PNCX_ITYPE_ULONGLONG, uint64_t, uint64_t, false, 0, 18446744073709551615ull,
          18446744073709551614ull)
#undef PNCX_IDEF

// ---------------------------------------------------------------------------
// byte order: the XDR external form is big-endian (SWAP2/4/8, ncx.m4:279-294)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint8_t bswap(uint8_t v) { return v; }
__device__ __forceinline__ uint16_t bswap(uint16_t v) { return __builtin_bswap16(v); }
__device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }
__device__ __forceinline__ uint64_t bswap(uint64_t v) { return __builtin_bswap64(v); }

template <typename T, typename U>
__device__ __forceinline__ T bits_to(U u) {
    static_assert(sizeof(T) == sizeof(U), "size");
    T t;
    __builtin_memcpy(&t, &u, sizeof t);
    return t;
}

// ---------------------------------------------------------------------------
// x86-64 gcc cast emulation.  cvttsd2si returns the
// "integer indefinite" value 0x80..0 for NaN and out-of-range inputs; narrow
// targets are converted through 32 bits, uint32 through 64 bits, and uint64
// through gcc's compare-with-2^63 sequence.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t cvtt_i32(double x) {
    return (x >= -2147483648.0 && x < 2147483648.0) ? (int32_t)x : INT32_MIN;
}
__device__ __forceinline__ int64_t cvtt_i64(double x) {
    return (x >= -9223372036854775808.0 && x < 9223372036854775808.0) ? (int64_t)x : INT64_MIN;
}
__device__ __forceinline__ uint64_t cvtt_u64(double x) {
    if (x >= 9223372036854775808.0)   // comisd 2^63; jnb (false for NaN)
        return (uint64_t)cvtt_i64(x - 9223372036854775808.0) ^ 0x8000000000000000ull;
    return (uint64_t)cvtt_i64(x);
}
// C cast (T)x of a floating value as compiled by gcc -O2 on x86-64
template <typename T>
__device__ __forceinline__ T x86_cast(double x) {
    if constexpr (std::is_same<T, int8_t>::value || std::is_same<T, uint8_t>::value ||
                  std::is_same<T, int16_t>::value || std::is_same<T, uint16_t>::value ||
                  std::is_same<T, int32_t>::value)
        return (T)cvtt_i32(x);
    else if constexpr (std::is_same<T, uint32_t>::value)
        return (T)cvtt_i64(x);
    else if constexpr (std::is_same<T, int64_t>::value)
        return cvtt_i64(x);
    else
        return cvtt_u64(x);
}

// cvtsd2ss / cvtss2sd: RNE value conversion; NaN keeps sign and the top
// payload bits and is quieted.
__device__ __forceinline__ float f64_to_f32(double x) {
    uint64_t b = bits_to<uint64_t>(x);
    if ((b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) {
        uint32_t r = ((uint32_t)(b >> 32) & 0x80000000u) | 0x7fc00000u |
                     (uint32_t)((b >> 29) & 0x3fffffu);
        return bits_to<float>(r);
    }
    return (float)x;
}
__device__ __forceinline__ double f32_to_f64(float x) {
    uint32_t b = bits_to<uint32_t>(x);
    if ((b & 0x7fffffffu) > 0x7f800000u) {
        uint64_t r = ((uint64_t)(b & 0x80000000u) << 32) | 0x7ff8000000000000ull |
                     ((uint64_t)(b & 0x3fffffu) << 29);
        return bits_to<double>(r);
    }
    return (double)x;
}

// exact integer range test (NCX_GET1I / NCX_PUT1I checks are exact)
template <typename S>
__device__ __forceinline__ bool in_range(S v, long long lo, unsigned long long hi) {
    if constexpr (std::is_signed<S>::value) {
        long long x = (long long)v;
        if (x < lo) return false;
        if (x < 0) return true;
        return (unsigned long long)x <= hi;
    } else {
        return (unsigned long long)v <= hi;
    }
}

// ---------------------------------------------------------------------------
// float (NC_FLOAT / itype float) -> integer on the float itself.  The
// reference widens to double and casts (NCX_GET1F / NCX_PUT1F, ncx.m4:
// 503-527, 604-625); for a float source both the range test and the x86 cast
// are decided exactly by the float's value, so the f64 detour (and, for the
// 64-bit targets, LLVM's f64 -> i64 expansion with its branches) is replaced
// by float compares and integer arithmetic on the bits.  Round 2 measured
// the detour at 66-70 % of peak for float <-> (u)int64 against 82-84 % for
// the other 4 <-> 8 byte pairs (profiles/r03a_pmc_pairs.txt: ~100 VALU and
// ~100 SALU instructions per wave, against 18 / 40 for NC_INT -> double).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool f32_isnan(uint32_t b) { return (b & 0x7fffffffu) > 0x7f800000u; }

// v_cvt_u32_f32: truncating, saturating, NaN -> 0 (a C cast of an
// out-of-range float is undefined, so the instruction is named)
__device__ __forceinline__ uint32_t hw_cvt_u32(float x) {
    uint32_t r;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// |trunc(x)| for a float with |x| < 2^64 (callers select other inputs away):
// the two 32-bit halves by exact float arithmetic and two hardware
// truncating converts -- |x| = hi * 2^32 + lo, where lo keeps a subset of
// x's 24 significant bits, so the fma is exact.  5 VALU against ~12 for
// shifting the mantissa by the exponent in 64 bits.  |x| = 2^64 gives
// hi = 0xffffffff, lo = 0.
__device__ __forceinline__ uint64_t f32_trunc_mag(float x) {
    const float xa = __builtin_fabsf(x);
    const uint32_t hi = hw_cvt_u32(xa * 0x1p-32f);
    const uint32_t lo = hw_cvt_u32(__builtin_fmaf(-(float)hi, 0x1p32f, xa));
    return ((uint64_t)hi << 32) | lo;
}

// x86_cast<T>((double)x) for a float x inside T's checked range or NaN,
// T of 8-32 bits (the 64-bit targets select on f32_trunc_mag in get1/put1)
template <typename T>
__device__ __forceinline__ T f32_cast(float x) {
    const uint32_t b = bits_to<uint32_t>(x);
    const bool nan = f32_isnan(b);
    const float xs = nan ? 0.0f : x;     // a C cast of NaN is undefined; of xs it is v_cvt_*_f32
    if constexpr (std::is_same<T, int8_t>::value || std::is_same<T, uint8_t>::value ||
                  std::is_same<T, int16_t>::value || std::is_same<T, uint16_t>::value) {
        // through cvtt_i32: NaN -> INT32_MIN, whose low 8/16 bits are 0
        return (T)(int32_t)xs;
    } else if constexpr (std::is_same<T, int32_t>::value) {
        return nan ? INT32_MIN : (int32_t)xs;
    } else {
        static_assert(std::is_same<T, uint32_t>::value, "64-bit targets: get1/put1 on the bits");
        return nan ? 0u : (uint32_t)xs;                        // through cvtt_i64: low half of INT64_MIN
    }
}

// d > hi || d < lo of GETF_CheckBND / NCX_PUT1F with d = (double)x, tested on
// the float: an upper bound that is not a float (2^31-1, 2^32-1) rounds up
// to the next power of two, and x > bound <=> x >= that power
template <long long LO, unsigned long long HI>
__device__ __forceinline__ bool f32_out_of_range(float x) {
    constexpr double hi = (double)HI, lo = (double)LO;
    constexpr float hf = (float)hi, lf = (float)lo;
    static_assert((double)lf == lo, "every lower bound (0, -2^7, -2^15, -2^31, -2^63) is a float");
    static_assert((double)hf >= hi, "an inexact upper bound rounds up to a power of two");
    return ((double)hf == hi ? x > hf : x >= hf) || x < lf;
}

template <typename T>
__device__ __forceinline__ double as_double(T v) {
    if constexpr (std::is_same<T, float>::value) return f32_to_f64(v);
    else return (double)v;
}

// ---------------------------------------------------------------------------
// GET: one external value (already byte-swapped to native) -> internal value
// ---------------------------------------------------------------------------
template <int XT, int IT>
__device__ __forceinline__ typename I<IT>::T get1(typename X<XT>::T xx, bool &bad) {
    using XI = X<XT>;
    using II = I<IT>;
    using IT_T = typename II::T;
    if constexpr (!XI::is_float && !II::is_float) {
        // NCX_GET1I (ncx.m4:560-598), NCX_GETN_BYTE (:2369-2392),
        // uchar->schar (:2817-2834): exact range test, fill = default of itype
        if (in_range(xx, II::lo, II::hi)) return (IT_T)xx;
        bad = true;
        return II::fill();
    } else if constexpr (!XI::is_float && II::is_float) {
        return (IT_T)xx;                        // int -> float/double (ncx.m4:551)
    } else if constexpr (XI::is_float && II::is_float) {
        if constexpr (XT == NC_FLOAT) {
            return f32_to_f64(xx);              // float -> double, exact (:546)
        } else {                                // get_NC_DOUBLE_float (:1834-1849)
            if (xx > 3.40282346638528859811704183484516925e+38 ||
                xx < -3.40282346638528859811704183484516925e+38) {
                bad = true;
                return II::fill();
            }
            return f64_to_f32(xx);
        }
    } else if constexpr (XT == NC_FLOAT) {
        // float -> integer without the double (f32_cast above), written as
        // selects (early returns became exec-mask branches: ~110 SALU per
        // wave); the same rules: GETF_CheckBND2 for (u)longlong (:518-527),
        // GETF_CheckBND + :511 for long, GETF_CheckBND (:503-513) otherwise
        const uint32_t b = bits_to<uint32_t>(xx);
        const bool nan = xx != xx;
        if constexpr (IT == PNCX_ITYPE_LONGLONG || IT == PNCX_ITYPE_LONG) {
            // |x| > 2^63 (not NaN): fill; +-2^63 exactly: INT64_MAX / INT64_MIN;
            // NaN: cvttsd2si's INT64_MIN.  Sign applied as (m ^ s) - s; -2^63
            // comes out as INT64_MIN by itself, +2^63 is one below it
            const bool o = __builtin_fabsf(xx) > 0x1p63f;
            const uint64_t s = (uint64_t)(int64_t)((int32_t)b >> 31);
            int64_t r = (int64_t)((f32_trunc_mag(xx) ^ s) - s);
            r = b == 0x5f000000u ? INT64_MAX : r;
            r = nan ? INT64_MIN : r;
            bad |= o;
            return o ? II::fill() : r;
        } else if constexpr (IT == PNCX_ITYPE_ULONGLONG) {
            // x > 2^64 or x < 0 (not -0, not NaN): fill; 2^64 exactly:
            // UINT64_MAX (hi is already all ones); NaN: 2^63 (cvtt_u64)
            const bool o = xx > 0x1p64f || xx < 0.0f;
            uint64_t r = f32_trunc_mag(xx);
            r = b == 0x5f800000u ? UINT64_MAX : r;
            r = nan ? 0x8000000000000000ull : r;
            bad |= o;
            return o ? II::fill() : r;
        } else {
            const bool o = f32_out_of_range<II::lo, II::hi>(xx);
            const IT_T r = f32_cast<IT_T>(xx);
            bad |= o;
            return o ? II::fill() : r;
        }
    } else {
        const double d = as_double(xx);
        if constexpr (IT == PNCX_ITYPE_LONGLONG) {             // GETF_CheckBND2 (:518-527)
            if (d == 9223372036854775808.0) return INT64_MAX;
            if (d == -9223372036854775808.0) return INT64_MIN;
            if (d > 9223372036854775808.0 || d < -9223372036854775808.0) { bad = true; return II::fill(); }
            return cvtt_i64(d);
        } else if constexpr (IT == PNCX_ITYPE_ULONGLONG) {
            if (d == 18446744073709551616.0) return UINT64_MAX;
            if (d > 18446744073709551616.0 || d < 0.0) { bad = true; return II::fill(); }
            return cvtt_u64(d);
        } else if constexpr (IT == PNCX_ITYPE_LONG) {          // GETF_CheckBND + :511
            if (d > 9223372036854775808.0 || d < -9223372036854775808.0) { bad = true; return II::fill(); }
            if (d == 9223372036854775808.0) return INT64_MAX;
            return cvtt_i64(d);
        } else {                                               // GETF_CheckBND (:503-513)
            const double hi = (double)II::hi;
            const double lo = (double)II::lo;
            if (d > hi || d < lo) { bad = true; return II::fill(); }
            return x86_cast<IT_T>(d);
        }
    }
}

// ---------------------------------------------------------------------------
// PUT: one internal value -> external value (native order; caller swaps)
//   fill: value written for out-of-range elements (the variable's fill value,
//   or the xtype default when fillp == NULL, NCX_PUT1I/PUT1F ncx.m4:610,642)
// ---------------------------------------------------------------------------
template <int XT, int IT>
__device__ __forceinline__ typename X<XT>::T put1(typename I<IT>::T v, typename X<XT>::T fill,
                                                  bool &bad) {
    using XI = X<XT>;
    using II = I<IT>;
    using XT_T = typename XI::T;
    if constexpr (!XI::is_float && !II::is_float) {
        // NCX_PUT1I (:631-665), NCX_PUTN_BYTE (:2561-2581) and the
        // hand-written <- schar/uchar codecs: exact range test
        if (in_range(v, XI::lo, XI::hi)) return (XT_T)v;
        bad = true;
        return fill;
    } else if constexpr (!XI::is_float && IT == PNCX_ITYPE_FLOAT) {
        // NCX_PUT1F (:604-625) / NCX_PUTN_BYTE from float, on the float
        // (f32_cast above), as selects; hi is 2^63 / 2^64 for the 64-bit
        // externals
        const bool o = f32_out_of_range<XI::lo, XI::hi>(v);
        XT_T r;
        if constexpr (XT == NC_INT64 || XT == NC_UINT64) {
            const uint32_t b = bits_to<uint32_t>(v);
            const uint64_t mag = f32_trunc_mag(v);
            if constexpr (XT == NC_INT64) {
                // |x| >= 2^63 and NaN: cvttsd2si's INT64_MIN (the larger ones
                // are out of range: fill below)
                const uint64_t s = (uint64_t)(int64_t)((int32_t)b >> 31);
                const int64_t sv = (int64_t)((mag ^ s) - s);
                r = !(__builtin_fabsf(v) < 0x1p63f) ? INT64_MIN : sv;
            } else {
                // cvtt_u64: 2^64 -> 0, NaN -> 2^63, [0, 2^64) exact
                uint64_t u = b == 0x5f800000u ? 0ull : mag;
                r = v != v ? 0x8000000000000000ull : u;
            }
        } else {
            r = f32_cast<XT_T>(v);
        }
        bad |= o;
        return o ? fill : r;
    } else if constexpr (!XI::is_float && II::is_float) {
        // NCX_PUT1F (:604-625) / NCX_PUTN_BYTE with a double itype
        const double d = as_double(v);
        const double hi = (double)XI::hi;     // 2^63 / 2^64 for the 64-bit ones
        const double lo = (double)XI::lo;
        if (d > hi || d < lo) { bad = true; return fill; }
        return x86_cast<XT_T>(d);
    } else if constexpr (XI::is_float && !II::is_float) {
        return (XT_T)v;                        // integer -> float/double, RNE
    } else if constexpr (XT == NC_FLOAT) {     // NCX_PUT1F(float, double) (:612)
        if (v > 3.40282346638528859811704183484516925e+38 ||
            v < -3.40282346638528859811704183484516925e+38) { bad = true; return fill; }
        return f64_to_f32(v);
    } else {                                   // put_NC_DOUBLE_float (:1871-1886)
        const double d = f32_to_f64(v);
        if (d > 1.7976931348623157e+308 || d < -1.7976931348623157e+308) { bad = true; return fill; }
        return d;
    }
}

// pairs whose reference codec writes nothing (1-byte externals) or swaps the
// bytes already in xbuf (ushort/uint <- schar, ncx.m4:818-841, 1036-1056)
// when fillp == NULL
template <int XT, int IT>
struct null_fill_preserves {
    static constexpr bool value =
        (XT == NC_BYTE || XT == NC_UBYTE) ||
        ((XT == NC_USHORT || XT == NC_UINT) && IT == PNCX_ITYPE_SCHAR);
};

}  // namespace pncx
