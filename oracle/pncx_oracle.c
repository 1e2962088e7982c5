/*
 * pncx_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of PnetCDF's XDR byte-swap and external<->internal NC type
 * conversion (the path this repository accelerates on MI355X).  It is the
 * CHECKER for the HIP path: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product library
 * (pnetcdf_amd/lib/libpncx.so) never links or calls it.
 *
 * Written from the semantics of the reference (PnetCDF 1.15.0), not from its
 * text.  Reference citations are to files under the PnetCDF tree:
 *   ncx.m4          = src/drivers/common/ncx.m4
 *   convert_swap.m4 = src/drivers/common/convert_swap.m4
 *   common.h        = src/drivers/include/common.h
 *   ncx_h.m4        = src/drivers/include/ncx_h.m4
 * Build assumptions are the reference defaults: ERANGE_FILL defined
 * (configure.ac:2436-2450, Makefile.am:28-29), little-endian x86-64, LP64,
 * gcc -O2.  Implementation-defined float->int casts (NaN, 2^63, 2^64) are
 * reproduced by using the very same C cast expressions the reference uses,
 * compiled by the same gcc on x86-64.
 *
 * Parity pinning: the reference's conversion code is m4 that needs GNU m4 and
 * configure-generated headers, neither of which this image has, so it cannot
 * be built here (DESIGN.md "Oracle").  This restatement is pinned instead by
 * the known answers recorded from the compiled reference in SURVEY.md §8(c)
 * and Appendix A.4, by the reference's own test expectations
 * (test/nc_test/util.c hash/inRange3/equal, test/testcases/test_erange.c,
 * test/testcases/erange_fill.m4) restated in tests/test_oracle_pinning.py,
 * and by the reference-held data fixture src/utils/ncmpidiff/tst_file.nc.
 */
#include <float.h>
#include <limits.h>
#include <stdint.h>
#include <string.h>

#include "../include/pncx.h"

typedef signed char        schar;
typedef unsigned char      uchar;
typedef unsigned short     ushort;
typedef unsigned int       uint;
typedef long long          longlong;
typedef unsigned long long ulonglong;

/* External limits, ncx_h.m4:81-106 */
#define X_SCHAR_MIN  (-128)
#define X_SCHAR_MAX  127
#define X_UCHAR_MAX  255U
#define X_SHORT_MIN  (-32768)
#define X_SHORT_MAX  32767
#define X_USHORT_MAX 65535U
#define X_INT_MIN    (-2147483647-1)
#define X_INT_MAX    2147483647
#define X_UINT_MAX   4294967295U
#define X_INT64_MIN  (-9223372036854775807LL-1LL)
#define X_INT64_MAX  9223372036854775807LL
#define X_UINT64_MAX 18446744073709551615ULL
#define X_FLOAT_MAX  3.402823466e+38f
#define X_FLOAT_MIN  (-X_FLOAT_MAX)
#define X_DOUBLE_MAX 1.7976931348623157e+308
#define X_DOUBLE_MIN (-X_DOUBLE_MAX)

/* ------------------------------------------------------------------------ */
/* Byte reversal: SWAP2/SWAP4/SWAP8 (ncx.m4:279-294)                         */
/* ------------------------------------------------------------------------ */
static inline uint16_t bs16(uint16_t a) { return (uint16_t)(((a & 0xff) << 8) | ((a >> 8) & 0xff)); }
static inline uint32_t bs32(uint32_t a)
{
    return (a << 24) | ((a << 8) & 0x00ff0000u) | ((a >> 8) & 0x0000ff00u) | (a >> 24);
}
static inline uint64_t bs64(uint64_t a)
{
    return ((a & 0x00000000000000FFULL) << 56) | ((a & 0x000000000000FF00ULL) << 40) |
           ((a & 0x0000000000FF0000ULL) << 24) | ((a & 0x00000000FF000000ULL) << 8) |
           ((a & 0x000000FF00000000ULL) >> 8)  | ((a & 0x0000FF0000000000ULL) >> 24) |
           ((a & 0x00FF000000000000ULL) >> 40) | ((a & 0xFF00000000000000ULL) >> 56);
}

/* ------------------------------------------------------------------------ */
/* Element decoders/encoders: get_ix_<T>/put_ix_<T>                          */
/* (short ncx.m4:695-716, ushort :783-804, int :898-935, uint :997-1019,     */
/*  float :1087-1105, double :1549-1567, int64 :1927-1949, uint64 :1999-2021) */
/* All are unaligned-safe (memcpy), like the reference.                     */
/* ------------------------------------------------------------------------ */
#define DEF_CODEC(NAME, CT, UT, BS)                                           \
    static inline CT dec_##NAME(const uchar *p)                               \
    { UT u; CT v; memcpy(&u, p, sizeof u); u = BS(u); memcpy(&v, &u, sizeof v); return v; } \
    static inline void enc_##NAME(uchar *p, CT v)                             \
    { UT u; memcpy(&u, &v, sizeof u); u = BS(u); memcpy(p, &u, sizeof u); }

#define BS8(a) (a)
DEF_CODEC(schar,  schar,     uint8_t,  BS8)
DEF_CODEC(uchar,  uchar,     uint8_t,  BS8)
DEF_CODEC(short,  short,     uint16_t, bs16)
DEF_CODEC(ushort, ushort,    uint16_t, bs16)
DEF_CODEC(int,    int,       uint32_t, bs32)
DEF_CODEC(uint,   uint,      uint32_t, bs32)
DEF_CODEC(float,  float,     uint32_t, bs32)
DEF_CODEC(double, double,    uint64_t, bs64)
DEF_CODEC(int64,  longlong,  uint64_t, bs64)
DEF_CODEC(uint64, ulonglong, uint64_t, bs64)

/* exact integer range test (the reference's NCX_GET1I/NCX_PUT1I checks,
 * ncx.m4:574-591, 644-657, are exact mathematical range tests) */
#define IN_RANGE(v, lo, hi) ((__int128)(v) >= (__int128)(lo) && (__int128)(v) <= (__int128)(hi))

/* ------------------------------------------------------------------------ */
/* In-place swap: ncmpii_in_swapn (convert_swap.m4:137-197)                  */
/* ------------------------------------------------------------------------ */
void orc_in_swapn(void *buf, long long nelems, int esize)
{
    size_t i;
    uchar *p = (uchar *)buf;
    if (esize <= 1 || nelems <= 0) return;                 /* :147 */
    if (esize == 4) {                                       /* :149-159 */
        for (i = 0; i < (size_t)nelems; i++) {
            uint32_t t; memcpy(&t, p + 4 * i, 4); t = bs32(t); memcpy(p + 4 * i, &t, 4);
        }
    } else if (esize == 8) {                                /* :160-174 */
        for (i = 0; i < (size_t)nelems; i++) {
            uint64_t t; memcpy(&t, p + 8 * i, 8); t = bs64(t); memcpy(p + 8 * i, &t, 8);
        }
    } else if (esize == 2) {                                /* :175-183 */
        for (i = 0; i < (size_t)nelems; i++) {
            uint16_t t; memcpy(&t, p + 2 * i, 2); t = bs16(t); memcpy(p + 2 * i, &t, 2);
        }
    } else {                                                /* :184-195 generic */
        long long k;
        for (k = 0; k < nelems; k++, p += esize) {
            for (i = 0; i < (size_t)esize / 2; i++) {
                uchar t = p[i]; p[i] = p[esize - 1 - i]; p[esize - 1 - i] = t;
            }
        }
    }
}

/* Out-of-place swap of n elements (swapn2b/4b/8b, ncx.m4:297-467). */
static void orc_swapn(void *dst, const void *src, long long n, int esize)
{
    if (dst != src) memmove(dst, src, (size_t)n * (size_t)esize);
    orc_in_swapn(dst, n, esize);
}

/* ------------------------------------------------------------------------ */
/* ncmpii_need_convert (convert_swap.m4:85-116) / NEED_BYTE_SWAP (common.h)  */
/* ------------------------------------------------------------------------ */
int orc_need_convert(int format, int xtype, int itype)
{
    if (xtype == NC_CHAR) return 0;                                   /* :90-93 */
    if (format < PNCX_FORMAT_CDF5 && xtype == NC_BYTE && itype == PNCX_ITYPE_UCHAR)
        return 0;                                                     /* :96-97 */
    if (itype == PNCX_ITYPE_LONG) itype = PNCX_ITYPE_LONGLONG;        /* :102 */
    return !((xtype == NC_BYTE   && itype == PNCX_ITYPE_SCHAR)    ||  /* :105-115 */
             (xtype == NC_SHORT  && itype == PNCX_ITYPE_SHORT)    ||
             (xtype == NC_INT    && itype == PNCX_ITYPE_INT)      ||
             (xtype == NC_FLOAT  && itype == PNCX_ITYPE_FLOAT)    ||
             (xtype == NC_DOUBLE && itype == PNCX_ITYPE_DOUBLE)   ||
             (xtype == NC_UBYTE  && itype == PNCX_ITYPE_UCHAR)    ||
             (xtype == NC_USHORT && itype == PNCX_ITYPE_USHORT)   ||
             (xtype == NC_UINT   && itype == PNCX_ITYPE_UINT)     ||
             (xtype == NC_INT64  && itype == PNCX_ITYPE_LONGLONG) ||
             (xtype == NC_UINT64 && itype == PNCX_ITYPE_ULONGLONG));
}

int orc_need_swap(int xtype, int itype)
{
    return ((xtype == NC_CHAR  && itype == PNCX_ITYPE_CHAR)  ||
            (xtype == NC_BYTE  && itype == PNCX_ITYPE_SCHAR) ||
            (xtype == NC_UBYTE && itype == PNCX_ITYPE_UCHAR)) ? 0 : 1;
}

/* ======================================================================== */
/* GET: external xtype -> internal itype                                     */
/*   Loop shape: NCX_GETN (ncx.m4:2480-2493): every element is converted,    */
/*   the first non-NOERR status is returned.                                 */
/* ======================================================================== */
#define DEF_GETN(XN, XCT, IN, ICT, BODY)                                      \
    __attribute__((unused)) static int getn_##XN##_##IN(const uchar *xp, uchar *ipb, long long n)     \
    {                                                                         \
        int status = NC_NOERR;                                                \
        long long k;                                                          \
        for (k = 0; k < n; k++, xp += sizeof(XCT), ipb += sizeof(ICT)) {      \
            XCT xx = dec_##XN(xp);                                            \
            ICT v;                                                            \
            int err = NC_NOERR;                                               \
            BODY                                                              \
            memcpy(ipb, &v, sizeof v);                                        \
            if (status == NC_NOERR) status = err;                             \
        }                                                                     \
        return status;                                                        \
    }

/* integer -> integer: NCX_GET1I (ncx.m4:560-598); fill = FillDefaultValue
 * of the INTERNAL type (ncx.m4:97-111; long -> NC_FILL_INT) */
#define G_I2I(ICT, LO, HI, FILL) \
    if (!IN_RANGE(xx, LO, HI)) { v = (ICT)(FILL); err = NC_ERANGE; } else v = (ICT)xx;
/* float/double -> integer: GETF_CheckBND (ncx.m4:503-513) */
#define G_F2I(ICT, HI_D, LO_D, FILL) \
    if (xx > (HI_D) || xx < (LO_D)) { v = (ICT)(FILL); err = NC_ERANGE; } else v = (ICT)xx;
/* float/double -> long: GETF_CheckBND with the LONG_MAX special (:511) */
#define G_F2LONG \
    if (xx > (double)LONG_MAX || xx < (double)LONG_MIN) { v = PNCX_FILL_INT; err = NC_ERANGE; } \
    else if (xx == (double)LONG_MAX) v = LONG_MAX; else v = (long)xx;
/* float/double -> longlong: GETF_CheckBND2 signed branch (ncx.m4:518-527) */
#define G_F2LL(XCT) \
    if (xx == (XCT)LLONG_MAX) v = LLONG_MAX; \
    else if (xx == LLONG_MIN) v = LLONG_MIN; \
    else if (xx > (double)LLONG_MAX || xx < (double)LLONG_MIN) { v = PNCX_FILL_INT64; err = NC_ERANGE; } \
    else v = (longlong)xx;
/* float/double -> ulonglong: GETF_CheckBND2 unsigned branch (:520) */
#define G_F2ULL(XCT) \
    if (xx == (XCT)ULLONG_MAX) v = ULLONG_MAX; \
    else if (xx > (double)ULLONG_MAX || xx < 0) { v = PNCX_FILL_UINT64; err = NC_ERANGE; } \
    else v = (ulonglong)xx;
/* plain cast: NCX_GET1F default branch (:551) / int->float (:546) */
#define G_CAST(ICT) v = (ICT)xx;
/* double -> float: get_NC_DOUBLE_float (ncx.m4:1834-1849) */
#define G_D2F \
    if (xx > FLT_MAX) { v = PNCX_FILL_FLOAT; err = NC_ERANGE; } \
    else if (xx < (-FLT_MAX)) { v = PNCX_FILL_FLOAT; err = NC_ERANGE; } \
    else v = (float)xx;
/* NC_BYTE -> unsigned itype: NCX_GETN_BYTE (ncx.m4:2369-2392) */
#define G_B2U(ICT, FILL) \
    if (xx < 0) { v = (ICT)(FILL); err = NC_ERANGE; } else v = (ICT)(signed)xx;
/* NC_UBYTE -> schar: hand-written ncx.m4:2817-2834 */
#define G_UB2SC \
    if (xx > SCHAR_MAX) { v = PNCX_FILL_BYTE; err = NC_ERANGE; } else v = (schar)xx;

/* integer internal types: ranges and default fills */
#define LIM_schar     SCHAR_MIN, SCHAR_MAX, PNCX_FILL_BYTE
#define LIM_uchar     0, UCHAR_MAX, PNCX_FILL_UBYTE
#define LIM_short     SHRT_MIN, SHRT_MAX, PNCX_FILL_SHORT
#define LIM_ushort    0, USHRT_MAX, PNCX_FILL_USHORT
#define LIM_int       INT_MIN, INT_MAX, PNCX_FILL_INT
#define LIM_uint      0, UINT_MAX, PNCX_FILL_UINT
#define LIM_long      LONG_MIN, LONG_MAX, PNCX_FILL_INT
#define LIM_longlong  LLONG_MIN, LLONG_MAX, PNCX_FILL_INT64
#define LIM_ulonglong 0, ULLONG_MAX, PNCX_FILL_UINT64
#define G_I2I_(ICT, ...) G_I2I(ICT, __VA_ARGS__)
#define GI(ICT) G_I2I_(ICT, LIM_##ICT)

/* float/double -> integer internal types (GETF_CheckBND arguments) */
#define FB_schar  (double)SCHAR_MAX, (double)SCHAR_MIN, PNCX_FILL_BYTE
#define FB_uchar  (double)UCHAR_MAX, 0, PNCX_FILL_UBYTE
#define FB_short  (double)SHRT_MAX, (double)SHRT_MIN, PNCX_FILL_SHORT
#define FB_ushort (double)USHRT_MAX, 0, PNCX_FILL_USHORT
#define FB_int    (double)INT_MAX, (double)INT_MIN, PNCX_FILL_INT
#define FB_uint   (double)UINT_MAX, 0, PNCX_FILL_UINT
#define G_F2I_(ICT, ...) G_F2I(ICT, __VA_ARGS__)
#define GF(ICT) G_F2I_(ICT, FB_##ICT)

/* The getn instantiation matrix mirrors ncx.m4:2743-3637. */
#define GET_FROM_INTEGER(XN, XCT)                                   \
    DEF_GETN(XN, XCT, schar, schar, GI(schar))                      \
    DEF_GETN(XN, XCT, uchar, uchar, GI(uchar))                      \
    DEF_GETN(XN, XCT, short, short, GI(short))                      \
    DEF_GETN(XN, XCT, ushort, ushort, GI(ushort))                   \
    DEF_GETN(XN, XCT, int, int, GI(int))                            \
    DEF_GETN(XN, XCT, uint, uint, GI(uint))                         \
    DEF_GETN(XN, XCT, long, long, GI(long))                         \
    DEF_GETN(XN, XCT, longlong, longlong, GI(longlong))             \
    DEF_GETN(XN, XCT, ulonglong, ulonglong, GI(ulonglong))          \
    DEF_GETN(XN, XCT, float, float, G_CAST(float))                  \
    DEF_GETN(XN, XCT, double, double, G_CAST(double))

GET_FROM_INTEGER(short,  short)        /* NCX_GET1I(short, *)  ncx.m4:718-728   */
GET_FROM_INTEGER(ushort, ushort)       /* NCX_GET1I(ushort, *) ncx.m4:806-816   */
GET_FROM_INTEGER(int,    int)          /* NCX_GET1I(int, *)    ncx.m4:937-949   */
GET_FROM_INTEGER(uint,   uint)         /* NCX_GET1I(uint, *)   ncx.m4:1021-1034 */
GET_FROM_INTEGER(int64,  longlong)     /* NCX_GET1I(int64, *)  ncx.m4:1951-1963 */
GET_FROM_INTEGER(uint64, ulonglong)    /* NCX_GET1I(uint64, *) ncx.m4:2023-2035 */

#define GET_FROM_FLOATING(XN, XCT)                                  \
    DEF_GETN(XN, XCT, schar, schar, GF(schar))                      \
    DEF_GETN(XN, XCT, uchar, uchar, GF(uchar))                      \
    DEF_GETN(XN, XCT, short, short, GF(short))                      \
    DEF_GETN(XN, XCT, ushort, ushort, GF(ushort))                   \
    DEF_GETN(XN, XCT, int, int, GF(int))                            \
    DEF_GETN(XN, XCT, uint, uint, GF(uint))                         \
    DEF_GETN(XN, XCT, long, long, G_F2LONG)                         \
    DEF_GETN(XN, XCT, longlong, longlong, G_F2LL(XCT))              \
    DEF_GETN(XN, XCT, ulonglong, ulonglong, G_F2ULL(XCT))

GET_FROM_FLOATING(float,  float)       /* NCX_GET1F(float, *)  ncx.m4:1503-1512 */
DEF_GETN(float, float, double, double, G_CAST(double))             /* :546  */
GET_FROM_FLOATING(double, double)      /* NCX_GET1F(double, *) ncx.m4:1824-1832 */
DEF_GETN(double, double, float, float, G_D2F)                       /* :1834 */

/* 1-byte externals: NCX_GETN_BYTE instantiations ncx.m4:2745-2849 */
DEF_GETN(schar, schar, uchar, uchar, G_B2U(uchar, PNCX_FILL_UBYTE))
DEF_GETN(schar, schar, short, short, G_CAST(short))
DEF_GETN(schar, schar, ushort, ushort, G_B2U(ushort, PNCX_FILL_USHORT))
DEF_GETN(schar, schar, int, int, G_CAST(int))
DEF_GETN(schar, schar, uint, uint, G_B2U(uint, PNCX_FILL_UINT))
DEF_GETN(schar, schar, long, long, G_CAST(long))
DEF_GETN(schar, schar, longlong, longlong, G_CAST(longlong))
DEF_GETN(schar, schar, ulonglong, ulonglong, G_B2U(ulonglong, PNCX_FILL_UINT64))
DEF_GETN(schar, schar, float, float, G_CAST(float))
DEF_GETN(schar, schar, double, double, G_CAST(double))
DEF_GETN(uchar, uchar, schar, schar, G_UB2SC)
DEF_GETN(uchar, uchar, short, short, G_CAST(short))
DEF_GETN(uchar, uchar, ushort, ushort, G_CAST(ushort))
DEF_GETN(uchar, uchar, int, int, G_CAST(int))
DEF_GETN(uchar, uchar, uint, uint, G_CAST(uint))
DEF_GETN(uchar, uchar, long, long, G_CAST(long))
DEF_GETN(uchar, uchar, longlong, longlong, G_CAST(longlong))
DEF_GETN(uchar, uchar, ulonglong, ulonglong, G_CAST(ulonglong))
DEF_GETN(uchar, uchar, float, float, G_CAST(float))
DEF_GETN(uchar, uchar, double, double, G_CAST(double))

/* ======================================================================== */
/* PUT: internal itype -> external xtype                                     */
/*   Loop shape: NCX_PUTN (ncx.m4:2688-2702).  The fill value written for an */
/*   out-of-range element is *fillp (native order, the variable's           */
/*   _FillValue or the xtype default, ncmpio_util.c:705-711); with           */
/*   fillp == NULL the multi-byte codecs write FillDefaultValue(xtype)       */
/*   (NCX_PUT1I/NCX_PUT1F initialise xx with it, ncx.m4:610,642).            */
/* ======================================================================== */
#define DEF_PUTN(XN, XCT, IN, ICT, XDEF, BODY)                                \
    __attribute__((unused)) static int putn_##XN##_##IN(uchar *xp, const uchar *ipb, long long n, \
                                const void *fillp)                            \
    {                                                                         \
        int status = NC_NOERR;                                                \
        long long k;                                                          \
        for (k = 0; k < n; k++, xp += sizeof(XCT), ipb += sizeof(ICT)) {      \
            ICT v;                                                            \
            XCT xx = (XCT)(XDEF);                                             \
            int err = NC_NOERR;                                               \
            (void)fillp;                                                      \
            memcpy(&v, ipb, sizeof v);                                        \
            BODY                                                              \
            enc_##XN(xp, xx);                                                 \
            if (status == NC_NOERR) status = err;                             \
        }                                                                     \
        return status;                                                        \
    }

#define PFILL(XCT) do { if (fillp != NULL) memcpy(&xx, fillp, sizeof(XCT)); err = NC_ERANGE; } while (0)
/* integer -> integer: NCX_PUT1I (ncx.m4:631-665) */
#define P_I2I(XCT, LO, HI) if (!IN_RANGE(v, LO, HI)) PFILL(XCT); else xx = (XCT)v;
/* float/double -> integer xtype: NCX_PUT1F (ncx.m4:604-625) */
#define P_F2I(XCT, HI_D, LO_D) if (v > (HI_D) || v < (LO_D)) PFILL(XCT); else xx = (XCT)v;
/* any -> float xtype without check (NCX_PUT1F for integer itypes, :620) */
#define P_CAST(XCT) xx = (XCT)v;
/* double -> NC_FLOAT: NCX_PUT1F(float, double) (:612) */
#define P_D2F if (v > (double)X_FLOAT_MAX || v < X_FLOAT_MIN) PFILL(float); else xx = (float)v;
/* float -> NC_DOUBLE: hand-written put_NC_DOUBLE_float (ncx.m4:1871-1886) */
#define P_F2D if ((double)(v) > X_DOUBLE_MAX || (double)(v) < X_DOUBLE_MIN) PFILL(double); else xx = (double)v;

#define XR_short  X_SHORT_MIN, X_SHORT_MAX
#define XR_ushort 0, X_USHORT_MAX
#define XR_int    X_INT_MIN, X_INT_MAX
#define XR_uint   0, X_UINT_MAX
#define XR_int64  X_INT64_MIN, X_INT64_MAX
#define XR_uint64 0, X_UINT64_MAX
#define XF_short  (double)X_SHORT_MAX, (double)X_SHORT_MIN
#define XF_ushort (double)X_USHORT_MAX, 0
#define XF_int    (double)X_INT_MAX, (double)X_INT_MIN
#define XF_uint   (double)X_UINT_MAX, 0
#define XF_int64  (double)X_INT64_MAX, (double)X_INT64_MIN
#define XF_uint64 (double)X_UINT64_MAX, 0
#define P_I2I_(XCT, ...) P_I2I(XCT, __VA_ARGS__)
#define P_F2I_(XCT, ...) P_F2I(XCT, __VA_ARGS__)

#define PUT_TO_INTEGER(XN, XCT, XDEF)                                        \
    DEF_PUTN(XN, XCT, schar, schar, XDEF, P_I2I_(XCT, XR_##XN))               \
    DEF_PUTN(XN, XCT, uchar, uchar, XDEF, P_I2I_(XCT, XR_##XN))               \
    DEF_PUTN(XN, XCT, short, short, XDEF, P_I2I_(XCT, XR_##XN))               \
    DEF_PUTN(XN, XCT, ushort, ushort, XDEF, P_I2I_(XCT, XR_##XN))             \
    DEF_PUTN(XN, XCT, int, int, XDEF, P_I2I_(XCT, XR_##XN))                   \
    DEF_PUTN(XN, XCT, uint, uint, XDEF, P_I2I_(XCT, XR_##XN))                 \
    DEF_PUTN(XN, XCT, long, long, XDEF, P_I2I_(XCT, XR_##XN))                 \
    DEF_PUTN(XN, XCT, longlong, longlong, XDEF, P_I2I_(XCT, XR_##XN))         \
    DEF_PUTN(XN, XCT, ulonglong, ulonglong, XDEF, P_I2I_(XCT, XR_##XN))       \
    DEF_PUTN(XN, XCT, float, float, XDEF, P_F2I_(XCT, XF_##XN))               \
    DEF_PUTN(XN, XCT, double, double, XDEF, P_F2I_(XCT, XF_##XN))

PUT_TO_INTEGER(short,  short,     PNCX_FILL_SHORT)    /* ncx.m4:730-759   */
PUT_TO_INTEGER(ushort, ushort,    PNCX_FILL_USHORT)   /* ncx.m4:818-860   */
PUT_TO_INTEGER(int,    int,       PNCX_FILL_INT)      /* ncx.m4:951-992   */
PUT_TO_INTEGER(uint,   uint,      PNCX_FILL_UINT)     /* ncx.m4:1036-1080 */
PUT_TO_INTEGER(int64,  longlong,  PNCX_FILL_INT64)    /* ncx.m4:1965-1977 */
PUT_TO_INTEGER(uint64, ulonglong, PNCX_FILL_UINT64)   /* ncx.m4:2037-2049 */

/* Hand-written put_NC_USHORT_schar (ncx.m4:818-841) and put_NC_UINT_schar
 * (:1036-1056): a negative value copies *fillp (native) and swaps it in
 * place; with fillp == NULL the bytes already in xbuf are swapped. */
#define DEF_PUTN_FROM_SCHAR(XN, XCT, BSF, UT)                                 \
    static int putn_##XN##_schar(uchar *xp, const uchar *ipb, long long n,    \
                                 const void *fillp)                           \
    {                                                                         \
        int status = NC_NOERR;                                                \
        long long k;                                                          \
        for (k = 0; k < n; k++, xp += sizeof(XCT), ipb++) {                   \
            schar v = (schar)ipb[0];                                          \
            if (v < 0) {                                                      \
                UT u;                                                         \
                if (fillp != NULL) memcpy(xp, fillp, sizeof(XCT));            \
                memcpy(&u, xp, sizeof u); u = BSF(u); memcpy(xp, &u, sizeof u); \
                if (status == NC_NOERR) status = NC_ERANGE;                   \
                continue;                                                     \
            }                                                                 \
            enc_##XN(xp, (XCT)v);                                             \
        }                                                                     \
        return status;                                                        \
    }
/* These replace the generic <- schar instances above in the dispatcher. */
static inline void enc_ushort_hw(uchar *p, ushort v) { enc_ushort(p, v); }
static inline void enc_uint_hw(uchar *p, uint v) { enc_uint(p, v); }
DEF_PUTN_FROM_SCHAR(ushort_hw, ushort, bs16, uint16_t)
DEF_PUTN_FROM_SCHAR(uint_hw,   uint,   bs32, uint32_t)

/* NC_FLOAT external (ncx.m4:1533-1542) */
#define PUT_TO_FLOAT_I(IN, ICT) DEF_PUTN(float, float, IN, ICT, PNCX_FILL_FLOAT, P_CAST(float))
PUT_TO_FLOAT_I(schar, schar)
PUT_TO_FLOAT_I(uchar, uchar)
PUT_TO_FLOAT_I(short, short)
PUT_TO_FLOAT_I(ushort, ushort)
PUT_TO_FLOAT_I(int, int)
PUT_TO_FLOAT_I(uint, uint)
PUT_TO_FLOAT_I(long, long)
PUT_TO_FLOAT_I(longlong, longlong)
PUT_TO_FLOAT_I(ulonglong, ulonglong)
DEF_PUTN(float, float, double, double, PNCX_FILL_FLOAT, P_D2F)

/* NC_DOUBLE external (ncx.m4:1861-1886) */
#define PUT_TO_DOUBLE_I(IN, ICT) DEF_PUTN(double, double, IN, ICT, PNCX_FILL_DOUBLE, P_CAST(double))
PUT_TO_DOUBLE_I(schar, schar)
PUT_TO_DOUBLE_I(uchar, uchar)
PUT_TO_DOUBLE_I(short, short)
PUT_TO_DOUBLE_I(ushort, ushort)
PUT_TO_DOUBLE_I(int, int)
PUT_TO_DOUBLE_I(uint, uint)
PUT_TO_DOUBLE_I(long, long)
PUT_TO_DOUBLE_I(longlong, longlong)
PUT_TO_DOUBLE_I(ulonglong, ulonglong)
DEF_PUTN(double, double, float, float, PNCX_FILL_DOUBLE, P_F2D)

/* 1-byte externals: NCX_PUTN_BYTE (ncx.m4:2561-2581), instantiations
 * :2779-2794 (schar) and :2889-2922 (uchar).  Out-of-range elements get
 * *fillp; with fillp == NULL the byte in xbuf is left untouched
 * (FillValue is a no-op, then SKIP_LOOP). */
#define DEF_PUTN_BYTE(XN, XCT, IN, ICT, BAD, CAST)                            \
    static int putn_##XN##_##IN(uchar *xp, const uchar *ipb, long long n,     \
                                const void *fillp)                            \
    {                                                                         \
        int status = NC_NOERR;                                                \
        long long k;                                                          \
        for (k = 0; k < n; k++, xp++, ipb += sizeof(ICT)) {                   \
            ICT v;                                                            \
            memcpy(&v, ipb, sizeof v);                                        \
            if (BAD) {                                                        \
                if (fillp != NULL) memcpy(xp, fillp, 1);                      \
                if (status == NC_NOERR) status = NC_ERANGE;                   \
                continue;                                                     \
            }                                                                 \
            { XCT xx = CAST; memcpy(xp, &xx, 1); }                            \
        }                                                                     \
        return status;                                                        \
    }

/* NC_BYTE <- itype: `*tp > (itype)X_SCHAR_MAX [|| *tp < X_SCHAR_MIN]`, cast (schar) */
DEF_PUTN_BYTE(schar, schar, uchar, uchar, v > (uchar)X_SCHAR_MAX, (schar)v)
DEF_PUTN_BYTE(schar, schar, short, short, v > (short)X_SCHAR_MAX || v < X_SCHAR_MIN, (schar)v)
DEF_PUTN_BYTE(schar, schar, ushort, ushort, v > (ushort)X_SCHAR_MAX, (schar)v)
DEF_PUTN_BYTE(schar, schar, int, int, v > (int)X_SCHAR_MAX || v < X_SCHAR_MIN, (schar)v)
DEF_PUTN_BYTE(schar, schar, uint, uint, v > (uint)X_SCHAR_MAX, (schar)v)
DEF_PUTN_BYTE(schar, schar, long, long, v > (long)X_SCHAR_MAX || v < X_SCHAR_MIN, (schar)v)
DEF_PUTN_BYTE(schar, schar, longlong, longlong, v > (longlong)X_SCHAR_MAX || v < X_SCHAR_MIN, (schar)v)
DEF_PUTN_BYTE(schar, schar, ulonglong, ulonglong, v > (ulonglong)X_SCHAR_MAX, (schar)v)
DEF_PUTN_BYTE(schar, schar, float, float, v > (float)X_SCHAR_MAX || v < X_SCHAR_MIN, (schar)v)
DEF_PUTN_BYTE(schar, schar, double, double, v > (double)X_SCHAR_MAX || v < X_SCHAR_MIN, (schar)v)
/* NC_UBYTE <- schar: hand-written ncx.m4:2889-2907 */
DEF_PUTN_BYTE(uchar, uchar, schar, schar, v < 0, (uchar)(signed)v)
/* NC_UBYTE <- itype: `*tp > (itype)X_UCHAR_MAX [|| *tp < 0]`, cast (uchar)[(signed)] */
DEF_PUTN_BYTE(uchar, uchar, short, short, v > (short)X_UCHAR_MAX || v < 0, (uchar)(signed)v)
DEF_PUTN_BYTE(uchar, uchar, ushort, ushort, v > (ushort)X_UCHAR_MAX, (uchar)v)
DEF_PUTN_BYTE(uchar, uchar, int, int, v > (int)X_UCHAR_MAX || v < 0, (uchar)(signed)v)
DEF_PUTN_BYTE(uchar, uchar, uint, uint, v > (uint)X_UCHAR_MAX, (uchar)v)
DEF_PUTN_BYTE(uchar, uchar, long, long, v > (long)X_UCHAR_MAX || v < 0, (uchar)(signed)v)
DEF_PUTN_BYTE(uchar, uchar, longlong, longlong, v > (longlong)X_UCHAR_MAX || v < 0, (uchar)(signed)v)
DEF_PUTN_BYTE(uchar, uchar, ulonglong, ulonglong, v > (ulonglong)X_UCHAR_MAX, (uchar)v)
DEF_PUTN_BYTE(uchar, uchar, float, float, v > (float)X_UCHAR_MAX || v < 0, (uchar)(signed)v)
DEF_PUTN_BYTE(uchar, uchar, double, double, v > (double)X_UCHAR_MAX || v < 0, (uchar)(signed)v)

/* ======================================================================== */
/* Dispatch: ncmpii_putn_NC_<X> / ncmpii_getn_NC_<X> (convert_swap.m4:202-330) */
/* ======================================================================== */
typedef int (*getn_fn)(const uchar *, uchar *, long long);
typedef int (*putn_fn)(uchar *, const uchar *, long long, const void *);

static int xsize(int xtype)
{
    switch (xtype) {
        case NC_BYTE: case NC_UBYTE: case NC_CHAR: return 1;
        case NC_SHORT: case NC_USHORT: return 2;
        case NC_INT: case NC_UINT: case NC_FLOAT: return 4;
        case NC_DOUBLE: case NC_INT64: case NC_UINT64: return 8;
        default: return -1;
    }
}

static int isize(int itype)
{
    switch (itype) {
        case PNCX_ITYPE_SCHAR: case PNCX_ITYPE_UCHAR: case PNCX_ITYPE_CHAR: return 1;
        case PNCX_ITYPE_SHORT: case PNCX_ITYPE_USHORT: return 2;
        case PNCX_ITYPE_INT: case PNCX_ITYPE_UINT: case PNCX_ITYPE_FLOAT: return 4;
        case PNCX_ITYPE_LONG: case PNCX_ITYPE_DOUBLE: case PNCX_ITYPE_LONGLONG:
        case PNCX_ITYPE_ULONGLONG: return 8;
        default: return -1;
    }
}

int orc_xlen(int xtype) { return xsize(xtype); }
int orc_ilen(int itype) { return isize(itype); }

/* 1 when the pair is a pure byte swap/copy (same representation) */
static int same_rep(int cdf_ver, int xtype, int itype)
{
    if (xtype == NC_BYTE && itype == PNCX_ITYPE_UCHAR && cdf_ver < 5) return 1; /* :219-222 */
    return !orc_need_convert(5, xtype, itype);
}

#define ROW_G(XN)                                                             \
    switch (itype) {                                                          \
        case PNCX_ITYPE_SCHAR: return getn_##XN##_schar;                      \
        case PNCX_ITYPE_UCHAR: return getn_##XN##_uchar;                      \
        case PNCX_ITYPE_SHORT: return getn_##XN##_short;                      \
        case PNCX_ITYPE_USHORT: return getn_##XN##_ushort;                    \
        case PNCX_ITYPE_INT: return getn_##XN##_int;                          \
        case PNCX_ITYPE_UINT: return getn_##XN##_uint;                        \
        case PNCX_ITYPE_LONG: return getn_##XN##_long;                        \
        case PNCX_ITYPE_FLOAT: return getn_##XN##_float;                      \
        case PNCX_ITYPE_DOUBLE: return getn_##XN##_double;                    \
        case PNCX_ITYPE_LONGLONG: return getn_##XN##_longlong;                \
        case PNCX_ITYPE_ULONGLONG: return getn_##XN##_ulonglong;              \
        default: return NULL;                                                 \
    }

/* same-type slots without an instance: never reached (same_rep first) */
#define getn_float_float NULL
#define getn_double_double NULL
#define getn_schar_schar NULL
#define getn_uchar_uchar NULL

static getn_fn get_fn(int xtype, int itype)
{
    switch (xtype) {
        case NC_BYTE:   ROW_G(schar)
        case NC_UBYTE:  ROW_G(uchar)
        case NC_SHORT:  ROW_G(short)
        case NC_USHORT: ROW_G(ushort)
        case NC_INT:    ROW_G(int)
        case NC_UINT:   ROW_G(uint)
        case NC_FLOAT:  ROW_G(float)
        case NC_DOUBLE: ROW_G(double)
        case NC_INT64:  ROW_G(int64)
        case NC_UINT64: ROW_G(uint64)
        default: return NULL;
    }
}

#define ROW_P(XN, SCHAR_FN)                                                   \
    switch (itype) {                                                          \
        case PNCX_ITYPE_SCHAR: return SCHAR_FN;                               \
        case PNCX_ITYPE_UCHAR: return putn_##XN##_uchar;                      \
        case PNCX_ITYPE_SHORT: return putn_##XN##_short;                      \
        case PNCX_ITYPE_USHORT: return putn_##XN##_ushort;                    \
        case PNCX_ITYPE_INT: return putn_##XN##_int;                          \
        case PNCX_ITYPE_UINT: return putn_##XN##_uint;                        \
        case PNCX_ITYPE_LONG: return putn_##XN##_long;                        \
        case PNCX_ITYPE_FLOAT: return putn_##XN##_float;                      \
        case PNCX_ITYPE_DOUBLE: return putn_##XN##_double;                    \
        case PNCX_ITYPE_LONGLONG: return putn_##XN##_longlong;                \
        case PNCX_ITYPE_ULONGLONG: return putn_##XN##_ulonglong;              \
        default: return NULL;                                                 \
    }

#define putn_schar_schar NULL
#define putn_uchar_uchar NULL
#define putn_float_float NULL
#define putn_double_double NULL

static putn_fn put_fn(int xtype, int itype)
{
    switch (xtype) {
        case NC_BYTE:   ROW_P(schar, putn_schar_schar)
        case NC_UBYTE:  ROW_P(uchar, putn_uchar_schar)
        case NC_SHORT:  ROW_P(short, putn_short_schar)
        case NC_USHORT: ROW_P(ushort, putn_ushort_hw_schar)
        case NC_INT:    ROW_P(int, putn_int_schar)
        case NC_UINT:   ROW_P(uint, putn_uint_hw_schar)
        case NC_FLOAT:  ROW_P(float, putn_float_schar)
        case NC_DOUBLE: ROW_P(double, putn_double_schar)
        case NC_INT64:  ROW_P(int64, putn_int64_schar)
        case NC_UINT64: ROW_P(uint64, putn_uint64_schar)
        default: return NULL;
    }
}

static int check_types(int xtype, int itype)
{
    if (xsize(xtype) < 0 || isize(itype) < 0) return NC_EBADTYPE;
    if ((xtype == NC_CHAR) != (itype == PNCX_ITYPE_CHAR)) return NC_ECHAR;
    return NC_NOERR;
}

/* ncmpii_getn_NC_<X>(cdf_ver, xbuf, ibuf, nelems, itype) */
int orc_getn(int cdf_ver, int xtype, const void *xbuf, void *ibuf,
             long long nelems, int itype)
{
    int err = check_types(xtype, itype);
    getn_fn f;
    if (err != NC_NOERR) return err;
    if (nelems <= 0) return NC_NOERR;
    if (xtype == NC_CHAR || same_rep(cdf_ver, xtype, itype)) {
        orc_swapn(ibuf, xbuf, nelems, xsize(xtype));   /* swapn / memcpy */
        return NC_NOERR;
    }
    f = get_fn(xtype, itype);
    if (f == NULL) return NC_EBADTYPE;
    return f((const uchar *)xbuf, (uchar *)ibuf, nelems);
}

/* ncmpii_putn_NC_<X>(cdf_ver, xbuf, ibuf, nelems, itype, fillp) */
int orc_putn(int cdf_ver, int xtype, void *xbuf, const void *ibuf,
             long long nelems, int itype, const void *fillp)
{
    int err = check_types(xtype, itype);
    putn_fn f;
    if (err != NC_NOERR) return err;
    if (nelems <= 0) return NC_NOERR;
    if (xtype == NC_CHAR || same_rep(cdf_ver, xtype, itype)) {
        orc_swapn(xbuf, ibuf, nelems, xsize(xtype));
        return NC_NOERR;
    }
    f = put_fn(xtype, itype);
    if (f == NULL) return NC_EBADTYPE;
    return f((uchar *)xbuf, (const uchar *)ibuf, nelems, fillp);
}
