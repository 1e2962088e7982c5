/*
 * pncx_ncmpii.c -- the reference-named conversion symbols (MPI-typed),
 * forwarding to the HIP-backed include/pncx.h entry points.
 * Drop-in for src/drivers/common/convert_swap.m4 (see include/pncx_ncmpii.h).
 */
#include <stdio.h>
#include <stdlib.h>

#include "../../include/pncx_ncmpii.h"

/* the itype switch of PUTN_XTYPE / GETN_XTYPE (convert_swap.m4:218-245) */
int pncx_itype_from_mpi(MPI_Datatype t)
{
    if (t == MPI_UNSIGNED_CHAR)      return PNCX_ITYPE_UCHAR;
    if (t == MPI_SIGNED_CHAR)        return PNCX_ITYPE_SCHAR;
    if (t == MPI_SHORT)              return PNCX_ITYPE_SHORT;
    if (t == MPI_UNSIGNED_SHORT)     return PNCX_ITYPE_USHORT;
    if (t == MPI_INT)                return PNCX_ITYPE_INT;
    if (t == MPI_UNSIGNED)           return PNCX_ITYPE_UINT;
    if (t == MPI_LONG)               return PNCX_ITYPE_LONG;
    if (t == MPI_FLOAT)              return PNCX_ITYPE_FLOAT;
    if (t == MPI_DOUBLE)             return PNCX_ITYPE_DOUBLE;
    if (t == MPI_LONG_LONG_INT)      return PNCX_ITYPE_LONGLONG;
    if (t == MPI_UNSIGNED_LONG_LONG) return PNCX_ITYPE_ULONGLONG;
    if (t == MPI_CHAR)               return PNCX_ITYPE_CHAR;
    return 0;
}

int ncmpii_need_convert(int format, int xtype, MPI_Datatype itype)
{
    return pncx_need_convert(format, xtype, pncx_itype_from_mpi(itype));
}

void ncmpii_in_swapn(void *buf, MPI_Offset nelems, int esize)
{
    int err = pncx_in_swapn(buf, (pncx_offset)nelems, esize);
    if (err != NC_NOERR) {
        /* the upstream signature is void: never return with the buffer
         * left unswapped */
        fprintf(stderr, "ncmpii_in_swapn: %s\n", pncx_strerror(err));
        abort();
    }
}

static int put(int cdf, int xtype, void *xbuf, const void *buf, MPI_Offset n,
               MPI_Datatype itype, void *fillp)
{
    const int it = pncx_itype_from_mpi(itype);
    if (it == 0) return NC_EBADTYPE;                       /* :245 */
    return pncx_putn(cdf, xtype, xbuf, buf, (pncx_offset)n, it, fillp);
}

static int get(int cdf, int xtype, const void *xbuf, void *buf, MPI_Offset n,
               MPI_Datatype itype)
{
    const int it = pncx_itype_from_mpi(itype);
    if (it == 0) return NC_EBADTYPE;                       /* :311 */
    return pncx_getn(cdf, xtype, xbuf, buf, (pncx_offset)n, it);
}

#define PUTN(X) \
    int ncmpii_putn_##X(void *xbuf, const void *buf, MPI_Offset n, MPI_Datatype t, void *fillp) \
    { return put(5, X, xbuf, buf, n, t, fillp); }
#define GETN(X) \
    int ncmpii_getn_##X(const void *xbuf, void *buf, MPI_Offset n, MPI_Datatype t) \
    { return get(5, X, xbuf, buf, n, t); }

PUTN(NC_UBYTE) PUTN(NC_SHORT) PUTN(NC_USHORT) PUTN(NC_INT) PUTN(NC_UINT)
PUTN(NC_FLOAT) PUTN(NC_DOUBLE) PUTN(NC_INT64) PUTN(NC_UINT64)
GETN(NC_UBYTE) GETN(NC_SHORT) GETN(NC_USHORT) GETN(NC_INT) GETN(NC_UINT)
GETN(NC_FLOAT) GETN(NC_DOUBLE) GETN(NC_INT64) GETN(NC_UINT64)

int ncmpii_putn_NC_BYTE(int cdf_ver, void *xbuf, const void *buf, MPI_Offset n,
                        MPI_Datatype t, void *fillp)
{
    return put(cdf_ver, NC_BYTE, xbuf, buf, n, t, fillp);
}

int ncmpii_getn_NC_BYTE(int cdf_ver, const void *xbuf, void *buf, MPI_Offset n, MPI_Datatype t)
{
    return get(cdf_ver, NC_BYTE, xbuf, buf, n, t);
}

int ncmpii_putn_NC_CHAR(void *xbuf, const void *buf, MPI_Offset n, MPI_Datatype t)
{
    return put(5, NC_CHAR, xbuf, buf, n, t, NULL);
}

int ncmpii_getn_NC_CHAR(const void *xbuf, void *buf, MPI_Offset n, MPI_Datatype t)
{
    return get(5, NC_CHAR, xbuf, buf, n, t);
}
