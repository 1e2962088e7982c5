/*
 * pncx_ncx.c -- the reference's ncx.h aggregate conversion interface
 * (include/pncx_ncx.h; src/drivers/include/ncx_h.m4:225-374) over the HIP
 * conversion path.  Every ncmpix_{getn,putn}_<xtype>_<itype> forwards to
 * pncx_getn / pncx_putn with CDF-5 semantics (the ncx layer has no CDF-1/2
 * NC_BYTE special case; ncmpii_*_NC_BYTE adds it one level up), then
 * advances *xpp as the reference does: nelems * xsize, rounded up to 4
 * bytes for the pad_ variants, whose padding is zero-filled on put
 * (NCX_PAD_GETN_BYTE/SHORT ncx.m4:2397-2424,2500-2523; NCX_PAD_PUTN_BYTE/
 * SHORT :2586-2615,2709-2735; the text/void bodies :2343-2364,2528-2555).
 * The header primitives (ncx.m4:2060-2330) are scalar big-endian byte
 * operations on the host, as in the reference's header codec.
 */
#include <stdint.h>
#include <string.h>

#include "../../include/pncx_ncx.h"

#ifndef NC_EINTOVERFLOW
#define NC_EINTOVERFLOW (-221)   /* pnetcdf.h.in:642 */
#endif

/* ------------------------------------------------------------------------ */
/* aggregate conversions                                                     */
/* ------------------------------------------------------------------------ */
static long long pad4(long long nbytes) { return nbytes % 4 ? nbytes + 4 - nbytes % 4 : nbytes; }

static int ncx_getn(int xtype, int itype, const void **xpp, MPI_Offset n, void *ip, int pad)
{
    long long nb;
    int st = NC_NOERR;
    if (n > 0) st = pncx_getn(5, xtype, *xpp, ip, (pncx_offset)n, itype);
    if (st != NC_NOERR && st != NC_ERANGE) return st;
    nb = n > 0 ? (long long)n * pncx_xlen(xtype) : 0;
    *xpp = (const char *)*xpp + (pad ? pad4(nb) : nb);
    return st;
}

static int ncx_putn(int xtype, int itype, void **xpp, MPI_Offset n, const void *ip, const void *fillp, int pad)
{
    long long nb;
    int st = NC_NOERR;
    char *xp;
    if (n > 0) st = pncx_putn(5, xtype, *xpp, ip, (pncx_offset)n, itype, fillp);
    if (st != NC_NOERR && st != NC_ERANGE) return st;
    nb = n > 0 ? (long long)n * pncx_xlen(xtype) : 0;
    xp = (char *)*xpp + nb;
    if (pad && pad4(nb) != nb) {                     /* memcpy(xp, nada, rndup) */
        memset(xp, 0, (size_t)(pad4(nb) - nb));
        xp += pad4(nb) - nb;
    }
    *xpp = xp;
    return st;
}

/* XT is the type name without its NC_ prefix (BYTE, ...): NC_BYTE is a
 * macro and would expand to its code before reaching the ## paste */
#define NCX_GET(OP, PAD, XT, TN, CT, IT)                                                      \
    int ncmpix_##OP##_NC_##XT##_##TN(const void **xpp, MPI_Offset nelems, CT *ip)             \
    { return ncx_getn(NC_##XT, IT, xpp, nelems, ip, PAD); }
#define NCX_PUT(OP, PAD, XT, TN, CT, IT)                                                      \
    int ncmpix_##OP##_NC_##XT##_##TN(void **xpp, MPI_Offset nelems, const CT *ip, void *fillp) \
    { return ncx_putn(NC_##XT, IT, xpp, nelems, ip, fillp, PAD); }

/* the itype list of ncx_h.m4:326-346 */
#define NCX_ITYPES(M, OP, PAD, XT)                                    \
    M(OP, PAD, XT, schar, signed char, PNCX_ITYPE_SCHAR)              \
    M(OP, PAD, XT, uchar, unsigned char, PNCX_ITYPE_UCHAR)            \
    M(OP, PAD, XT, short, short, PNCX_ITYPE_SHORT)                    \
    M(OP, PAD, XT, ushort, unsigned short, PNCX_ITYPE_USHORT)         \
    M(OP, PAD, XT, int, int, PNCX_ITYPE_INT)                          \
    M(OP, PAD, XT, uint, unsigned int, PNCX_ITYPE_UINT)               \
    M(OP, PAD, XT, long, long, PNCX_ITYPE_LONG)                       \
    M(OP, PAD, XT, float, float, PNCX_ITYPE_FLOAT)                    \
    M(OP, PAD, XT, double, double, PNCX_ITYPE_DOUBLE)                 \
    M(OP, PAD, XT, longlong, long long, PNCX_ITYPE_LONGLONG)          \
    M(OP, PAD, XT, ulonglong, unsigned long long, PNCX_ITYPE_ULONGLONG)

/* external types with padded variants (BYTE, UBYTE, SHORT, USHORT) */
#define NCX_PADDED(XT)                                  \
    NCX_ITYPES(NCX_GET, getn, 0, XT)                    \
    NCX_ITYPES(NCX_GET, pad_getn, 1, XT)                \
    NCX_ITYPES(NCX_PUT, putn, 0, XT)                    \
    NCX_ITYPES(NCX_PUT, pad_putn, 1, XT)
#define NCX_UNPADDED(XT)                                \
    NCX_ITYPES(NCX_GET, getn, 0, XT)                    \
    NCX_ITYPES(NCX_PUT, putn, 0, XT)

NCX_PADDED(BYTE)
NCX_PADDED(UBYTE)
NCX_PADDED(SHORT)
NCX_PADDED(USHORT)
NCX_UNPADDED(INT)
NCX_UNPADDED(UINT)
NCX_UNPADDED(FLOAT)
NCX_UNPADDED(DOUBLE)
NCX_UNPADDED(INT64)
NCX_UNPADDED(UINT64)

/* text and opaque bytes: NC_CHAR copies through the same kernels */
int ncmpix_getn_text(const void **xpp, MPI_Offset n, char *cp) { return ncx_getn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, cp, 0); }
int ncmpix_pad_getn_text(const void **xpp, MPI_Offset n, char *cp) { return ncx_getn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, cp, 1); }
int ncmpix_putn_text(void **xpp, MPI_Offset n, const char *cp) { return ncx_putn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, cp, NULL, 0); }
int ncmpix_pad_putn_text(void **xpp, MPI_Offset n, const char *cp) { return ncx_putn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, cp, NULL, 1); }
int ncmpix_getn_void(const void **xpp, MPI_Offset n, void *vp) { return ncx_getn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, vp, 0); }
int ncmpix_pad_getn_void(const void **xpp, MPI_Offset n, void *vp) { return ncx_getn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, vp, 1); }
int ncmpix_putn_void(void **xpp, MPI_Offset n, const void *vp) { return ncx_putn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, vp, NULL, 0); }
int ncmpix_pad_putn_void(void **xpp, MPI_Offset n, const void *vp) { return ncx_putn(NC_CHAR, PNCX_ITYPE_CHAR, xpp, n, vp, NULL, 1); }

/* ------------------------------------------------------------------------ */
/* header primitives (ncx.m4:2060-2330)                                      */
/* ------------------------------------------------------------------------ */
static uint32_t be32(const void *p)
{
    const unsigned char *b = (const unsigned char *)p;
    return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
}
static uint64_t be64(const void *p) { return (uint64_t)be32(p) << 32 | be32((const char *)p + 4); }
static void put_be32(void *p, uint32_t v)
{
    unsigned char *b = (unsigned char *)p;
    b[0] = (unsigned char)(v >> 24); b[1] = (unsigned char)(v >> 16); b[2] = (unsigned char)(v >> 8); b[3] = (unsigned char)v;
}
static void put_be64(void *p, uint64_t v) { put_be32(p, (uint32_t)(v >> 32)); put_be32((char *)p + 4, (uint32_t)v); }

/* 32-bit unsigned (X_SIZEOF_SIZE_T = 4) */
int ncmpix_get_size_t(const void **xpp, size_t *ulp)
{
    *ulp = be32(*xpp);
    *xpp = (const char *)*xpp + 4;
    return NC_NOERR;
}

int ncmpix_put_size_t(void **xpp, const size_t *ulp)
{
    put_be32(*xpp, (uint32_t)*ulp);
    *xpp = (char *)*xpp + 4;
    return NC_NOERR;
}

int ncmpix_get_off_t(const void **xpp, off_t *lp, size_t sizeof_off_t)
{
    if (sizeof_off_t == 4) *lp = (off_t)(int32_t)be32(*xpp);
    else *lp = (off_t)(int64_t)be64(*xpp);
    *xpp = (const char *)*xpp + sizeof_off_t;
    return NC_NOERR;
}

int ncmpix_put_off_t(void **xpp, const off_t *lp, size_t sizeof_off_t)
{
    if (*lp < 0) return NC_ERANGE;                   /* no negative offsets */
    if (sizeof_off_t == 4) {
        if (*lp > 2147483647) return NC_EINTOVERFLOW;
        put_be32(*xpp, (uint32_t)*lp);
    } else {
        put_be64(*xpp, (uint64_t)*lp);
    }
    *xpp = (char *)*xpp + sizeof_off_t;
    return NC_NOERR;
}

int ncmpix_get_uint32(const void **xpp, unsigned int *ip)
{
    *ip = be32(*xpp);
    *xpp = (const char *)*xpp + 4;
    return NC_NOERR;
}

int ncmpix_get_uint64(const void **xpp, unsigned long long *ip)
{
    *ip = be64(*xpp);
    *xpp = (const char *)*xpp + 8;
    return NC_NOERR;
}

int ncmpix_put_uint32(void **xpp, const unsigned int ip)
{
    put_be32(*xpp, ip);
    *xpp = (char *)*xpp + 4;
    return NC_NOERR;
}

int ncmpix_put_uint64(void **xpp, const unsigned long long ip)
{
    put_be64(*xpp, ip);
    *xpp = (char *)*xpp + 8;
    return NC_NOERR;
}

int ncmpix_getn_uint32(const void **xpp, unsigned int *ip, int nelems)
{
    int i;
    for (i = 0; i < nelems; i++) ip[i] = be32((const char *)*xpp + 4 * (size_t)i);
    *xpp = (const char *)*xpp + 4 * (long long)nelems;
    return NC_NOERR;
}

int ncmpix_getn_uint64(const void **xpp, unsigned long long *ip, int nelems)
{
    int i;
    for (i = 0; i < nelems; i++) ip[i] = be64((const char *)*xpp + 8 * (size_t)i);
    *xpp = (const char *)*xpp + 8 * (long long)nelems;
    return NC_NOERR;
}

int ncmpix_putn_uint32(void **xpp, const unsigned int *ip, int nelems)
{
    int i;
    for (i = 0; i < nelems; i++) put_be32((char *)*xpp + 4 * (size_t)i, ip[i]);
    *xpp = (char *)*xpp + 4 * (long long)nelems;
    return NC_NOERR;
}

int ncmpix_putn_uint64(void **xpp, const unsigned long long *ip, int nelems)
{
    int i;
    for (i = 0; i < nelems; i++) put_be64((char *)*xpp + 8 * (size_t)i, ip[i]);
    *xpp = (char *)*xpp + 8 * (long long)nelems;
    return NC_NOERR;
}
