/*
 * pncx_nc.h -- file-level C-ABI over the MI355X conversion path.
 *
 * The callers either side of the hot path: the classic
 * CDF-1/2/5 header codec and file layout, blocking and nonblocking
 * put/get of subarrays, and the fill path.  Each entry point restates the
 * ncmpi_* API of the same name (src/include/pnetcdf.h.in) as implemented by
 * the ncmpio driver (struct PNC_driver, src/include/dispatch.h:63-125) for
 * one process on POSIX I/O:
 *
 *   pncx_nc_create / open / close / sync       ncmpi_create/open/close/sync
 *                                              (dispatchers/file.c, ncmpio_create.c, ncmpio_open.c,
 *                                               ncmpio_close.c:60-200)
 *   pncx_nc_redef / enddef / _enddef          ncmpio_enddef.c:1119-1351, NC_begins :359-612
 *   pncx_nc_def_dim / def_var / put_att ...   dispatchers/dimension.c, variable.c, attribute.c
 *   pncx_nc_set_fill / def_var_fill /
 *     fill_var_rec                             ncmpio_fill.c:620-848
 *   pncx_nc_put_varm / get_varm               ncmpi_{put,get}_var{,1,a,s,m}_<type>[_all]
 *                                              (dispatchers/var_getput.m4, ncmpio_getput.m4:106-473)
 *   pncx_nc_iput_varm / iget_varm / wait_all  ncmpi_i{put,get}_var*, ncmpi_wait_all
 *                                              (ncmpio_i_getput.m4:137-624, ncmpio_wait.c:587-808)
 *   pncx_nc_inq_file_format                   dispatchers/file.c:2023-2125
 *   pncx_nc_validate                          utils/ncvalidator (strict header padding)
 *
 * Data conversion goes through the HIP kernels (pncx.h); there is no CPU
 * conversion path: without a GPU, data calls and numeric attribute calls
 * return PNCX_EDEVICE.  Header-only operations (define mode, text
 * attributes, open/inquire/validate) do not need a GPU.
 *
 * Buffer layouts follow the reference:
 *   - start == NULL and count == NULL: the whole variable (ncmpi_put_var);
 *   - count == NULL: one element at start (var1);
 *   - stride == NULL: unit strides (vara);
 *   - imap == NULL: the user buffer is contiguous in C order (vars), else
 *     imap[d] is the element distance of dimension d in the buffer (varm).
 * itype is a PNCX_ITYPE_* (pncx.h); NC_ECHAR when exactly one of itype and
 * the variable's type is text.
 */
#ifndef PNCX_NC_H
#define PNCX_NC_H

#include "pncx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- modes and formats (pnetcdf.h.in:151-230, 578-615) ---- */
#define NC_NOWRITE        0x0000
#define NC_WRITE          0x0001
#define NC_CLOBBER        0x0000
#define NC_NOCLOBBER      0x0004
#define NC_64BIT_DATA     0x0020
#define NC_CLASSIC_MODEL  0x0100
#define NC_64BIT_OFFSET   0x0200
#define NC_NETCDF4        0x1000
#define NC_FILL           0
#define NC_NOFILL         0x100
#define NC_UNLIMITED      0L
#define NC_GLOBAL         (-1)
#define NC_REQ_NULL       (-1)
#define NC_REQ_ALL        (-1)
#define NC_GET_REQ_ALL    (-2)
#define NC_PUT_REQ_ALL    (-3)
#define NC_MAX_NAME       256
#define NC_FORMAT_UNKNOWN (-1)
#define NC_FORMAT_NETCDF4 3
#define NC_FORMAT_NETCDF4_CLASSIC 4
#define NC_FORMAT_CDF2    2
#define NC_FORMAT_CDF5    5

/* ---- errors (pnetcdf.h.in:400-640) ---- */
#define NC_EBADID         (-33)
#define NC_EEXIST         (-35)
#define NC_EPERM          (-37)
#define NC_ENOTINDEFINE   (-38)
#define NC_EINDEFINE      (-39)
#define NC_EINVALCOORDS   (-40)
#define NC_EMAXDIMS       (-41)
#define NC_ENAMEINUSE     (-42)
#define NC_ENOTATT        (-43)
#define NC_EMAXATTS       (-44)
#define NC_EBADDIM        (-46)
#define NC_EUNLIMPOS      (-47)
#define NC_EMAXVARS       (-48)
#define NC_ENOTVAR        (-49)
#define NC_EGLOBAL        (-50)
#define NC_ENOTNC         (-51)
#define NC_EMAXNAME       (-53)
#define NC_EUNLIMIT       (-54)
#define NC_EEDGE          (-57)
#define NC_ESTRIDE        (-58)
#define NC_EBADNAME       (-59)
#define NC_EVARSIZE       (-62)
#define NC_EDIMSIZE       (-63)
#define NC_ENOTNC3        (-113)
#define NC_ENOTBUILT      (-128)
#define NC_ENULLPAD       (-134)
#define NC_EFILE          (-204)
#define NC_EREAD          (-205)
#define NC_EWRITE         (-206)
#define NC_ENEGATIVECNT   (-210)
#define NC_EINVAL_REQUEST (-212)
#define NC_EPREVATTACHBUF (-216)
#define NC_ENULLABUF      (-217)
#define NC_EPENDINGBPUT   (-218)
#define NC_EINSUFFBUF     (-219)
#define NC_ENOENT         (-220)
#define NC_EINTOVERFLOW   (-221)
#define NC_ENULLSTART     (-226)
#define NC_EINVAL_CMODE   (-228)
#define NC_ESTRICTCDF2    (-232)
#define NC_ENOTRECVAR     (-233)
#define NC_ENOTFILL       (-234)
#define NC_EINVAL_OMODE   (-235)
#define NC_EPENDING       (-236)

/* ---- files ---- */
int pncx_nc_inq_file_format(const char *path, int *format);
int pncx_nc_create(const char *path, int cmode, int *ncid);
int pncx_nc_open(const char *path, int omode, int *ncid);
/* ncvalidator: decode the header with null-padding checks on.  Returns the
 * first fatal error, else NC_ENULLPAD if any padding is not null, else
 * NC_NOERR. */
int pncx_nc_validate(const char *path);
int pncx_nc_redef(int ncid);
int pncx_nc_enddef(int ncid);
int pncx_nc__enddef(int ncid, pncx_offset h_minfree, pncx_offset v_align,
                    pncx_offset v_minfree, pncx_offset r_align);
int pncx_nc_sync(int ncid);
int pncx_nc_close(int ncid);
/* Multi-process use: every rank opens the file and writes disjoint records;
 * the application reduces numrecs (max) and rank 0 records it here before
 * close (ncmpio_write_numrecs, ncmpio_util.c). */
int pncx_nc_sync_numrecs(int ncid, pncx_offset numrecs);
/* One file shared by several processes (the ncmpi_* driver on a
 * communicator, one process per GPU).  Every process keeps its own copy of
 * the header and runs the same define-mode calls; only the writer (rank 0)
 * writes header bytes and numrecs, moves data at enddef and fills new
 * variables, as the reference writes them from the root
 * (ncmpio_enddef.c:681, ncmpio_sync.c).  The caller orders the processes:
 * the writer creates (truncates) the file before the others open it with
 * pncx_nc_create_shared(writer = 0), and enddef/close are followed by a
 * barrier.  pncx_nc_set_numrecs raises this handle's numrecs (the MAX of
 * ncmpio_getput.m4:289-311) without writing it. */
int pncx_nc_create_shared(const char *path, int cmode, int writer, int *ncid);
int pncx_nc_set_writer(int ncid, int writer);
int pncx_nc_set_numrecs(int ncid, pncx_offset numrecs);

/* ---- define mode ---- */
int pncx_nc_def_dim(int ncid, const char *name, pncx_offset len, int *dimid);
int pncx_nc_def_var(int ncid, const char *name, int xtype, int ndims, const int *dimids, int *varid);
int pncx_nc_rename_dim(int ncid, int dimid, const char *name);
int pncx_nc_rename_var(int ncid, int varid, const char *name);
int pncx_nc_set_fill(int ncid, int fillmode, int *old_mode);
/* fill_value: one value of the variable's type in native byte order, or NULL */
int pncx_nc_def_var_fill(int ncid, int varid, int no_fill, const void *fill_value);
int pncx_nc_inq_var_fill(int ncid, int varid, int *no_fill, void *fill_value);
int pncx_nc_fill_var_rec(int ncid, int varid, pncx_offset recno);

/* ---- attributes (varid NC_GLOBAL for global attributes) ---- */
int pncx_nc_put_att(int ncid, int varid, const char *name, int xtype, pncx_offset nelems,
                    const void *buf, int itype);
int pncx_nc_get_att(int ncid, int varid, const char *name, void *buf, int itype);
int pncx_nc_del_att(int ncid, int varid, const char *name);
int pncx_nc_rename_att(int ncid, int varid, const char *name, const char *newname);

/* ---- inquiry ---- */
int pncx_nc_inq(int ncid, int *ndims, int *nvars, int *ngatts, int *unlimdimid);
int pncx_nc_inq_format(int ncid, int *format);
int pncx_nc_inq_dim(int ncid, int dimid, char *name, pncx_offset *len);
int pncx_nc_inq_dimid(int ncid, const char *name, int *dimid);
int pncx_nc_inq_var(int ncid, int varid, char *name, int *xtype, int *ndims, int *dimids, int *natts);
int pncx_nc_inq_varid(int ncid, const char *name, int *varid);
int pncx_nc_inq_varoffset(int ncid, int varid, pncx_offset *offset);
int pncx_nc_inq_att(int ncid, int varid, const char *name, int *xtype, pncx_offset *nelems);
int pncx_nc_inq_attname(int ncid, int varid, int attnum, char *name);
int pncx_nc_inq_header_size(int ncid, pncx_offset *size);
int pncx_nc_inq_header_extent(int ncid, pncx_offset *extent);
int pncx_nc_inq_recsize(int ncid, pncx_offset *recsize);
/* bytes moved by data calls since open: {put, get} (ncmpi_inq_put_size/get_size) */
int pncx_nc_inq_io_size(int ncid, pncx_offset *put_size, pncx_offset *get_size);

/* ---- blocking data access ---- */
int pncx_nc_put_varm(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                     const pncx_offset *stride, const pncx_offset *imap, const void *buf, int itype);
int pncx_nc_get_varm(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                     const pncx_offset *stride, const pncx_offset *imap, void *buf, int itype);
/* device-resident user buffer (HBM); conversion runs in HBM, the packed
 * external bytes cross PCIe once */
int pncx_nc_put_varm_dev(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                         const pncx_offset *stride, const pncx_offset *imap, const void *dbuf,
                         int itype, pncx_stream_t stream);
int pncx_nc_get_varm_dev(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                         const pncx_offset *stride, const pncx_offset *imap, void *dbuf,
                         int itype, pncx_stream_t stream);

/* ---- nonblocking: posted requests are converted and written together at
 * wait time (one batched conversion launch, offset-sorted coalesced I/O) ---- */
int pncx_nc_iput_varm(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                      const pncx_offset *stride, const pncx_offset *imap, const void *buf,
                      int itype, int *reqid);
int pncx_nc_iget_varm(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                      const pncx_offset *stride, const pncx_offset *imap, void *buf,
                      int itype, int *reqid);
/* varn: num subarrays (starts[i], counts[i]; counts or counts[i] NULL = one
 * element) of one variable, packed one after another in buf
 * (ncmpi_{put,get,iput,iget}_varn, dispatchers/var_getput.m4:426-560,
 * ncmpio_varn.m4:38-60).  A varn request is one request id; the blocking
 * calls are the nonblocking ones followed by a wait, as in the reference. */
int pncx_nc_put_varn(int ncid, int varid, int num, const pncx_offset *const *starts,
                     const pncx_offset *const *counts, const void *buf, int itype);
int pncx_nc_get_varn(int ncid, int varid, int num, const pncx_offset *const *starts,
                     const pncx_offset *const *counts, void *buf, int itype);
int pncx_nc_iput_varn(int ncid, int varid, int num, const pncx_offset *const *starts,
                      const pncx_offset *const *counts, const void *buf, int itype, int *reqid);
int pncx_nc_iget_varn(int ncid, int varid, int num, const pncx_offset *const *starts,
                      const pncx_offset *const *counts, void *buf, int itype, int *reqid);
/* buffered puts (ncmpi_buffer_attach / bput_var* / buffer_detach,
 * ncmpio_bput.c, ncmpio_i_getput.m4:266-310): the data are converted into the
 * attached buffer when posted, so the caller may reuse its buffer at once;
 * wait_all only writes.  Space is the external size of each request; it is
 * released at wait (tail first, as abuf_coalesce, ncmpio_wait.c:37-56). */
int pncx_nc_buffer_attach(int ncid, pncx_offset bufsize);
int pncx_nc_buffer_detach(int ncid);
int pncx_nc_inq_buffer_size(int ncid, pncx_offset *size);
int pncx_nc_inq_buffer_usage(int ncid, pncx_offset *usage);
int pncx_nc_bput_varm(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                      const pncx_offset *stride, const pncx_offset *imap, const void *buf,
                      int itype, int *reqid);
int pncx_nc_bput_varn(int ncid, int varid, int num, const pncx_offset *const *starts,
                      const pncx_offset *const *counts, const void *buf, int itype, int *reqid);
/* flexible API (ncmpi_{put,get,iput,iget}_varm[_all] with bufcount + an MPI
 * derived buftype, dispatchers/var_getput.m4:312-382, ncmpio_getput.m4:136-
 * 235): the user buffer is `bufcount` copies of a committed flattened
 * buftype (pncx.h pncx_type_commit; include/pncx_ncmpii.h flattens an
 * MPI_Datatype).  The pack/unpack runs fused into the conversion kernel.
 * buftype NULL plays MPI_DATATYPE_NULL (bufcount ignored, the buffer holds
 * the variable's own type).  bufcount == 0 returns NC_NOERR at once
 * (var_getput.m4:382); an element count that differs from the request's is
 * NC_EIOMISMATCH.  A nonblocking request keeps a reference to the buftype
 * until it completes, so the caller may free it after posting. */
int pncx_nc_put_varm_flex(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                          const pncx_offset *stride, const pncx_offset *imap, const void *buf,
                          pncx_offset bufcount, const pncx_dtype *buftype);
int pncx_nc_get_varm_flex(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                          const pncx_offset *stride, const pncx_offset *imap, void *buf,
                          pncx_offset bufcount, const pncx_dtype *buftype);
int pncx_nc_put_varm_flex_dev(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                              const pncx_offset *stride, const pncx_offset *imap, const void *dbuf,
                              pncx_offset bufcount, const pncx_dtype *buftype, pncx_stream_t stream);
int pncx_nc_get_varm_flex_dev(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                              const pncx_offset *stride, const pncx_offset *imap, void *dbuf,
                              pncx_offset bufcount, const pncx_dtype *buftype, pncx_stream_t stream);
int pncx_nc_iput_varm_flex(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                           const pncx_offset *stride, const pncx_offset *imap, const void *buf,
                           pncx_offset bufcount, const pncx_dtype *buftype, int *reqid);
int pncx_nc_iget_varm_flex(int ncid, int varid, const pncx_offset *start, const pncx_offset *count,
                           const pncx_offset *stride, const pncx_offset *imap, void *buf,
                           pncx_offset bufcount, const pncx_dtype *buftype, int *reqid);
/* nreqs == NC_REQ_ALL / NC_PUT_REQ_ALL / NC_GET_REQ_ALL: every pending (put/get) request */
int pncx_nc_wait_all(int ncid, int nreqs, int *reqids, int *statuses);
int pncx_nc_cancel(int ncid, int nreqs, int *reqids, int *statuses);
int pncx_nc_inq_nreqs(int ncid, int *nreqs);

#ifdef __cplusplus
}
#endif
#endif /* PNCX_NC_H */
