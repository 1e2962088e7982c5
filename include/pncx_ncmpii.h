/*
 * pncx_ncmpii.h -- reference-named, MPI-typed entry points of the
 * conversion layer, exported by libpncx_ncmpii.so (built against the MPI
 * headers the PnetCDF build uses).  Signatures are exactly those of
 * src/drivers/include/common.h:147-221; semantics are those of
 * src/drivers/common/convert_swap.m4.  Each forwards to include/pncx.h,
 * i.e. to the HIP kernels.  Linking this library in place of the
 * reference's convert_swap.o is the drop-in.
 *
 * Error behaviour follows the reference, with one addition: a HIP failure
 * (no GPU, launch error) is reported as PNCX_EDEVICE from the putn/getn
 * functions and aborts in ncmpii_in_swapn (which returns void upstream),
 * so a missing device can never silently skip the byte swap.
 */
#ifndef PNCX_NCMPII_H
#define PNCX_NCMPII_H

#include <mpi.h>
#include "pncx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* convert_swap.m4:85-116 */
int  ncmpii_need_convert(int format, int xtype, MPI_Datatype itype);
/* convert_swap.m4:137-197 */
void ncmpii_in_swapn(void *buf, MPI_Offset nelems, int esize);

/* convert_swap.m4:202-264 (PUTN_XTYPE) */
int ncmpii_putn_NC_CHAR  (void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_putn_NC_BYTE  (int cdf_ver, void *xbuf, const void *buf, MPI_Offset nelems,
                          MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_UBYTE (void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_SHORT (void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_USHORT(void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_INT   (void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_UINT  (void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_FLOAT (void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_DOUBLE(void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_INT64 (void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);
int ncmpii_putn_NC_UINT64(void *xbuf, const void *buf, MPI_Offset nelems, MPI_Datatype itype, void *fillp);

/* convert_swap.m4:270-330 (GETN_XTYPE) */
int ncmpii_getn_NC_CHAR  (const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_BYTE  (int cdf_ver, const void *xbuf, void *buf, MPI_Offset nelems,
                          MPI_Datatype itype);
int ncmpii_getn_NC_UBYTE (const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_SHORT (const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_USHORT(const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_INT   (const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_UINT  (const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_FLOAT (const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_DOUBLE(const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_INT64 (const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);
int ncmpii_getn_NC_UINT64(const void *xbuf, void *buf, MPI_Offset nelems, MPI_Datatype itype);

/* MPI itype -> enum pncx_itype (0 if not a conversion itype) */
int pncx_itype_from_mpi(MPI_Datatype itype);

#ifdef __cplusplus
}
#endif
#endif
