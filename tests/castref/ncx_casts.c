/*
 * ncx_casts.c -- TEST INFRASTRUCTURE ONLY: the reference's float->integer
 * conversion expressions, written out as plain C (not copied) so that gcc
 * -O2 on this host compiles them exactly as the reference's x86-64 build
 * compiles ncx.m4.  A second, compiled source of truth for the x86
 * implementation-defined edges (NaN -> unsigned, (long long)2^63,
 * (unsigned long long)NaN) beside oracle/pncx_oracle.c and
 * tests/golden/known_answers.json (VERDICT r04 "Next" 7).
 *
 * get (x_get_<xtype>_<itype>, ncx.m4:537-554 NCX_GET1F with ERANGE_FILL):
 *   xtype float/double, itype other than long long / unsigned long long /
 *   double (and float from float): GETF_CheckBND, ncx.m4:503-513:
 *       if (xx > (double)ITYPE_MAX || xx < Dmin(itype)) -> fill, NC_ERANGE
 *       else *ip = (itype)xx         (Dmin = 0 for unsigned, else (double)MIN)
 *   itype long long / unsigned long long: GETF_CheckBND2, ncx.m4:518-527:
 *       if (xx == (xtype)MAX) *ip = MAX; [signed: else if (xx == MIN) *ip = MIN;]
 *       else if (xx > (double)MAX || xx < Dmin) -> fill, NC_ERANGE
 *       else *ip = (itype)xx
 * put (x_put_<xtype>_<itype>, ncx.m4:604-625 NCX_PUT1F, ERANGE_FILL):
 *   itype double: if (*ip > (double)X_MAX || *ip < DXmin) -> fill, NC_ERANGE
 *                 else xx = (ix_xtype)*ip
 *   itype float:  the same with FXmin ((double)X_MIN for signed, 0 unsigned)
 *
 * Output: one line per (dir, src, dst, input): the result's bits in hex and
 * the status (0 or -60), for the host's gcc to answer.
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define NC_ERANGE (-60)
/* the itype fill values (ERANGE_FILL's FillDefaultValue, netcdf.h NC_FILL_*) */
#define FILL_SCHAR ((signed char)-127)
#define FILL_UCHAR ((unsigned char)255)
#define FILL_SHORT ((short)-32767)
#define FILL_USHORT ((unsigned short)65535)
#define FILL_INT (-2147483647)
#define FILL_UINT (4294967295U)
#define FILL_INT64 ((long long)-9223372036854775806LL)
#define FILL_UINT64 (18446744073709551614ULL)

static void out(const char *dir, const char *s, const char *d, double in, unsigned long long bits, int st)
{
    unsigned long long ib;
    memcpy(&ib, &in, 8);
    printf("%s %s %s %016llx %llx %d\n", dir, s, d, ib, bits, st);
}

/* GETF_CheckBND for a narrow/32-bit integer itype from double xx */
#define GET_BND(XT, NAME, T, TMAX, DMIN, FILL, U)                                 \
    static void get_##XT##_##NAME(XT xx, double in)                              \
    {                                                                          \
        T v;                                                                   \
        int st = 0;                                                            \
        if (xx > (double)TMAX || xx < (DMIN)) { v = FILL; st = NC_ERANGE; }    \
        else v = (T)xx;                                                        \
        out("get", #XT, #NAME, in, (unsigned long long)(U)v, st);              \
    }
GET_BND(double, schar, signed char, SCHAR_MAX, (double)SCHAR_MIN, FILL_SCHAR, unsigned char)
GET_BND(double, uchar, unsigned char, UCHAR_MAX, 0, FILL_UCHAR, unsigned char)
GET_BND(double, short, short, SHRT_MAX, (double)SHRT_MIN, FILL_SHORT, unsigned short)
GET_BND(double, ushort, unsigned short, USHRT_MAX, 0, FILL_USHORT, unsigned short)
GET_BND(double, int, int, INT_MAX, (double)INT_MIN, FILL_INT, unsigned int)
GET_BND(double, uint, unsigned int, UINT_MAX, 0, FILL_UINT, unsigned int)
GET_BND(float, schar, signed char, SCHAR_MAX, (double)SCHAR_MIN, FILL_SCHAR, unsigned char)
GET_BND(float, uchar, unsigned char, UCHAR_MAX, 0, FILL_UCHAR, unsigned char)
GET_BND(float, short, short, SHRT_MAX, (double)SHRT_MIN, FILL_SHORT, unsigned short)
GET_BND(float, ushort, unsigned short, USHRT_MAX, 0, FILL_USHORT, unsigned short)
GET_BND(float, int, int, INT_MAX, (double)INT_MIN, FILL_INT, unsigned int)
GET_BND(float, uint, unsigned int, UINT_MAX, 0, FILL_UINT, unsigned int)

/* GETF_CheckBND2 for long long / unsigned long long */
#define GET_BND2_S(XT)                                                         \
    static void get_##XT##_longlong(XT xx, double in)                          \
    {                                                                          \
        long long v;                                                           \
        int st = 0;                                                            \
        if (xx == (XT)LLONG_MAX) v = LLONG_MAX;                                \
        else if (xx == LLONG_MIN) v = LLONG_MIN;                               \
        else if (xx > (double)LLONG_MAX || xx < (double)LLONG_MIN) { v = FILL_INT64; st = NC_ERANGE; } \
        else v = (long long)xx;                                                \
        out("get", #XT, "longlong", in, (unsigned long long)v, st);            \
    }
#define GET_BND2_U(XT)                                                         \
    static void get_##XT##_ulonglong(XT xx, double in)                         \
    {                                                                          \
        unsigned long long v;                                                  \
        int st = 0;                                                            \
        if (xx == (XT)ULLONG_MAX) v = ULLONG_MAX;                              \
        else if (xx > (double)ULLONG_MAX || xx < 0) { v = FILL_UINT64; st = NC_ERANGE; } \
        else v = (unsigned long long)xx;                                       \
        out("get", #XT, "ulonglong", in, v, st);                               \
    }
GET_BND2_S(double)
GET_BND2_U(double)
GET_BND2_S(float)
GET_BND2_U(float)

/* NCX_PUT1F into the 8-byte integer xtypes (the A.4 (long long)2^63 edge) */
static void put_int64_double(double ip)
{
    long long xx = FILL_INT64;
    int st = 0;
    if (ip > (double)LLONG_MAX || ip < (double)LLONG_MIN) st = NC_ERANGE;
    else xx = (long long)ip;
    out("put", "double", "int64", ip, (unsigned long long)xx, st);
}
static void put_uint64_double(double ip)
{
    unsigned long long xx = FILL_UINT64;
    int st = 0;
    if (ip > (double)ULLONG_MAX || ip < 0) st = NC_ERANGE;
    else xx = (unsigned long long)ip;
    out("put", "double", "uint64", ip, xx, st);
}
static void put_int_double(double ip)
{
    int xx = FILL_INT;
    int st = 0;
    if (ip > (double)INT_MAX || ip < (double)INT_MIN) st = NC_ERANGE;
    else xx = (int)ip;
    out("put", "double", "int", ip, (unsigned long long)(unsigned int)xx, st);
}
static void put_uint_double(double ip)
{
    unsigned int xx = FILL_UINT;
    int st = 0;
    if (ip > (double)UINT_MAX || ip < 0) st = NC_ERANGE;
    else xx = (unsigned int)ip;
    out("put", "double", "uint", ip, (unsigned long long)xx, st);
}

int main(void)
{
    /* volatile: the inputs reach the casts at run time, as file data does */
    static volatile double ins[] = {
        0.0, -0.0, 1.5, -1.5, -0.5, 0.99999, 127.5, 128.0, -128.5, -129.0, 255.9, 256.0,
        32767.9, 32768.0, -32768.9, -32769.0, 65535.5, 65536.0,
        2147483647.0, 2147483647.5, 2147483648.0, -2147483648.0, -2147483648.9, -2147483649.0,
        4294967295.0, 4294967295.9, 4294967296.0,
        9223372036854775808.0 /* 2^63 */, -9223372036854775808.0, 9223372036854774784.0 /* 2^63 - 1024 */,
        18446744073709551616.0 /* 2^64 */, 18446744073709549568.0 /* 2^64 - 2048 */,
        1e300, -1e300, DBL_MAX, -DBL_MAX, 3.4028234663852886e38 /* FLT_MAX */, 4.9e-324, -4.9e-324};
    const size_t n = sizeof ins / sizeof ins[0];
    double specials[5];
    size_t i, k;
    specials[0] = NAN;
    specials[1] = -NAN;
    specials[2] = INFINITY;
    specials[3] = -INFINITY;
    {   /* a NaN with a payload */
        unsigned long long b = 0x7ff8000000012345ULL;
        memcpy(&specials[4], &b, 8);
    }
    for (k = 0; k < n + 5; k++) {
        const double in = k < n ? ins[k] : specials[k - n];
        const float fin = (float)in;
        volatile double vd = in;
        volatile float vf = fin;
        get_double_schar(vd, in); get_double_uchar(vd, in); get_double_short(vd, in);
        get_double_ushort(vd, in); get_double_int(vd, in); get_double_uint(vd, in);
        get_double_longlong(vd, in); get_double_ulonglong(vd, in);
        /* a float source: the input rounded to float (its own bits printed) */
        get_float_schar(vf, (double)fin); get_float_uchar(vf, (double)fin); get_float_short(vf, (double)fin);
        get_float_ushort(vf, (double)fin); get_float_int(vf, (double)fin); get_float_uint(vf, (double)fin);
        get_float_longlong(vf, (double)fin); get_float_ulonglong(vf, (double)fin);
        put_int64_double(vd); put_uint64_double(vd); put_int_double(vd); put_uint_double(vd);
    }
    (void)i;
    return 0;
}
