/*
 * pncx_mpi.h -- MPI-datatype side of the flexible API, exported by
 * libpncx_mpi.so (linked against the MPI library the PnetCDF build uses).
 *
 * The reference's flexible calls take (buf, bufcount, MPI_Datatype buftype)
 * with any derived datatype of one element type (ncmpii_buftype_decode,
 * src/drivers/common/dtype_decode.c:628-694) and MPI_Pack / MPI_Unpack it
 * around the conversion (ncmpio_util.c:620-652, 889-933).  Here the
 * datatype is flattened once into its typemap -- runs of elements in pack
 * order -- and committed (pncx.h pncx_type_commit); the pack then runs
 * fused into the conversion kernel.  The decode walks the combiners the
 * reference's ncmpii_dtype_decode walks (dtype_decode.c:198-399): named,
 * dup, contiguous, (h)vector, (h)indexed, (h)indexed_block, struct,
 * subarray, resized; any other combiner (darray, f90) is flattened by
 * packing offset planes with MPI_Pack itself.
 *
 * MPI must be initialised.  Errors follow the reference: NC_EMULTITYPES
 * for a datatype mixing element types, NC_EBADTYPE for an element type the
 * conversion has no itype for (MPI_BYTE, MPI_LONG_DOUBLE, ...).
 */
#ifndef PNCX_MPI_H
#define PNCX_MPI_H

#include <mpi.h>
#include "pncx.h"
#include "pncx_nc.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef NC_COUNT_IGNORE
#define NC_COUNT_IGNORE (-1)     /* pnetcdf.h.in:583 */
#endif

/* Flatten `buftype` into nblocks runs: blocklen[i] elements of *itype at byte
 * displacement disp[i] from the buffer origin, in MPI_Pack order; *extent =
 * the MPI extent (distance between consecutive copies).  Adjacent runs are
 * merged.  *disp and *blocklen are malloc'ed (free with free()). */
int pncx_mpi_type_flatten(MPI_Datatype buftype, int *itype, MPI_Offset *nblocks, MPI_Offset **disp,
                          MPI_Offset **blocklen, MPI_Offset *extent);
/* flatten + pncx_type_commit */
int pncx_mpi_type_commit(MPI_Datatype buftype, pncx_dtype **dtype);

/* The flexible ncmpi_{put,get,iput,iget}_varm (pnetcdf.h.in flexible API;
 * var / var1 / vara / vars are the NULL-argument cases, pncx_nc.h).
 * bufcount == NC_COUNT_IGNORE: buftype must be a predefined type (the
 * high-level API, var_getput.m4:366-377, NC_EINVAL otherwise);
 * buftype == MPI_DATATYPE_NULL: the buffer holds the variable's own type. */
int pncx_ncmpi_put_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                        const MPI_Offset *stride, const MPI_Offset *imap, const void *buf,
                        MPI_Offset bufcount, MPI_Datatype buftype);
int pncx_ncmpi_get_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                        const MPI_Offset *stride, const MPI_Offset *imap, void *buf,
                        MPI_Offset bufcount, MPI_Datatype buftype);
int pncx_ncmpi_iput_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                         const MPI_Offset *stride, const MPI_Offset *imap, const void *buf,
                         MPI_Offset bufcount, MPI_Datatype buftype, int *reqid);
int pncx_ncmpi_iget_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                         const MPI_Offset *stride, const MPI_Offset *imap, void *buf,
                         MPI_Offset bufcount, MPI_Datatype buftype, int *reqid);

#ifdef __cplusplus
}
#endif
#endif /* PNCX_MPI_H */
