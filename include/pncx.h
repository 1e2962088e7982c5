/*
 * pncx.h -- C-ABI of the MI355X-native XDR byte-swap + NC type-conversion path.
 *
 * This is the drop-in boundary for PnetCDF's per-element conversion layer.
 * Every entry point below replaces one reference interface; the reference
 * location is cited next to it (paths relative to the PnetCDF 1.15.0 tree).
 * The exact reference-named symbols (ncmpii_in_swapn, ncmpii_putn_NC_<X>,
 * ncmpii_getn_NC_<X>, ncmpii_need_convert, taking MPI_Datatype) are exported
 * by the MPI-typed shim declared in include/pncx_ncmpii.h, which forwards to
 * the functions here.
 *
 * Plain C: no HIP, torch or MPI types appear in any signature.  Buffers are
 * plain pointers, element counts are 64-bit (MPI_Offset), streams are opaque
 * (a hipStream_t passed as void*).  Host-buffer entry points stage through
 * HBM and run the HIP kernels; there is no CPU conversion path.
 */
#ifndef PNCX_H
#define PNCX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* NetCDF external types (src/include/pnetcdf.h.in:66-83)                    */
/* ------------------------------------------------------------------------ */
#ifndef NC_BYTE
#define NC_NAT     0
#define NC_BYTE    1
#define NC_CHAR    2
#define NC_SHORT   3
#define NC_INT     4
#define NC_FLOAT   5
#define NC_DOUBLE  6
#define NC_UBYTE   7
#define NC_USHORT  8
#define NC_UINT    9
#define NC_INT64  10
#define NC_UINT64 11
#endif

/* Status codes (src/include/pnetcdf.h.in:400,442,461,479) */
#ifndef NC_NOERR
#define NC_NOERR      0
#define NC_EINVAL   (-36)
#define NC_EBADTYPE (-45)
#define NC_ECHAR    (-56)
#define NC_ERANGE   (-60)
#define NC_ENOMEM   (-61)
#endif
/* pncx-specific: a HIP runtime call failed (no device, launch error, ...) */
#define PNCX_EDEVICE (-1900)

/* CDF format numbers (src/include/pnetcdf.h.in:214-227) */
#ifndef NC_FORMAT_CLASSIC
#define NC_FORMAT_CLASSIC      1
#define NC_FORMAT_64BIT_OFFSET 2
#define NC_FORMAT_64BIT_DATA   5
#endif
#define PNCX_FORMAT_CDF1 1
#define PNCX_FORMAT_CDF2 2
#define PNCX_FORMAT_CDF5 5

/* Default fill values (src/include/pnetcdf.h.in:104-114) */
#define PNCX_FILL_BYTE   ((signed char)-127)
#define PNCX_FILL_CHAR   ((char)0)
#define PNCX_FILL_SHORT  ((short)-32767)
#define PNCX_FILL_INT    (-2147483647)
#define PNCX_FILL_FLOAT  (9.9692099683868690e+36f)
#define PNCX_FILL_DOUBLE (9.9692099683868690e+36)
#define PNCX_FILL_UBYTE  (255)
#define PNCX_FILL_USHORT (65535)
#define PNCX_FILL_UINT   (4294967295U)
#define PNCX_FILL_INT64  ((long long)-9223372036854775806LL)
#define PNCX_FILL_UINT64 ((unsigned long long)18446744073709551614ULL)

/* MPI_Offset equivalent (64-bit signed) */
typedef long long pncx_offset;

/*
 * Internal (in-memory) element types: one per MPI datatype accepted by the
 * itype switch of ncmpii_putn_NC_<X>/ncmpii_getn_NC_<X>
 * (src/drivers/common/convert_swap.m4:218-245, 285-311).  LONG is the LP64
 * 8-byte long: same bits as LONGLONG but it keeps its own get-side fill value
 * (NC_FILL_INT, ncx.m4:104).
 */
enum pncx_itype {
    PNCX_ITYPE_SCHAR     = 1,   /* MPI_SIGNED_CHAR        */
    PNCX_ITYPE_UCHAR     = 2,   /* MPI_UNSIGNED_CHAR      */
    PNCX_ITYPE_SHORT     = 3,   /* MPI_SHORT              */
    PNCX_ITYPE_USHORT    = 4,   /* MPI_UNSIGNED_SHORT     */
    PNCX_ITYPE_INT       = 5,   /* MPI_INT                */
    PNCX_ITYPE_UINT      = 6,   /* MPI_UNSIGNED           */
    PNCX_ITYPE_LONG      = 7,   /* MPI_LONG (LP64)        */
    PNCX_ITYPE_FLOAT     = 8,   /* MPI_FLOAT              */
    PNCX_ITYPE_DOUBLE    = 9,   /* MPI_DOUBLE             */
    PNCX_ITYPE_LONGLONG  = 10,  /* MPI_LONG_LONG_INT      */
    PNCX_ITYPE_ULONGLONG = 11,  /* MPI_UNSIGNED_LONG_LONG */
    PNCX_ITYPE_CHAR      = 12   /* MPI_CHAR (text only)   */
};

/* Direction of a conversion segment. */
enum pncx_dir {
    PNCX_PUT = 1,   /* internal (user) -> external (XDR big-endian), putn */
    PNCX_GET = 2    /* external -> internal, getn */
};

/* Opaque stream handle: a hipStream_t (NULL = the null stream). */
typedef void *pncx_stream_t;

/* ------------------------------------------------------------------------ */
/* Type metadata                                                             */
/* ------------------------------------------------------------------------ */

/* ncmpii_xlen_nc_type (src/drivers/common/utils.c:46-62): external size,
 * or -1 for an unknown type. */
int pncx_xlen(int xtype);
/* sizeof the internal type (LP64), or -1 for an unknown itype. */
int pncx_ilen(int itype);

/* ncmpii_need_convert (src/drivers/common/convert_swap.m4:85-116):
 * 1 if a type cast is needed between xtype and itype in CDF format
 * `format` (1, 2 or 5), 0 if only a byte swap (or nothing) is needed. */
int pncx_need_convert(int format, int xtype, int itype);

/* NEED_BYTE_SWAP (src/drivers/include/common.h:47-54): 0 for the three
 * 1-byte same-type pairs, 1 otherwise (little-endian host). */
int pncx_need_swap(int xtype, int itype);

/* ------------------------------------------------------------------------ */
/* Host-buffer entry points (drop-in semantics)                              */
/*   Buffers are caller-owned host memory, any alignment.  Data is staged    */
/*   through HBM and converted by the HIP kernels.                           */
/* ------------------------------------------------------------------------ */

/* ncmpii_in_swapn (convert_swap.m4:137-197; proto common.h:150-151):
 * in-place byte reversal of nelems elements of esize bytes.  No-op when
 * esize <= 1 or nelems <= 0.  Returns NC_NOERR or PNCX_EDEVICE. */
int pncx_in_swapn(void *buf, pncx_offset nelems, int esize);

/* ncmpii_putn_NC_<X> (convert_swap.m4:202-264; proto common.h:153-186):
 * convert nelems elements of itype from ibuf into external type xtype at
 * xbuf (big-endian).  cdf_ver matters only for xtype NC_BYTE (CDF-1/2 treat
 * NC_BYTE<-uchar as a raw copy, convert_swap.m4:219-222).  fillp points to
 * the fill value of xtype in native byte order (ncmpio_util.c:705-711), or
 * NULL (then the reference's NULL-fill behaviour is reproduced).
 * Returns NC_NOERR, NC_ERANGE (non-fatal; all elements are converted,
 * out-of-range ones are filled, ncx.m4:2693-2698), NC_EBADTYPE,
 * NC_ECHAR or PNCX_EDEVICE. */
int pncx_putn(int cdf_ver, int xtype, void *xbuf, const void *ibuf,
              pncx_offset nelems, int itype, const void *fillp);

/* ncmpii_getn_NC_<X> (convert_swap.m4:270-330; proto common.h:188-221):
 * convert nelems external elements at xbuf into itype at ibuf.  Out-of-range
 * elements receive the default fill value of itype (ncx.m4:97-111) and the
 * call returns NC_ERANGE. */
int pncx_getn(int cdf_ver, int xtype, const void *xbuf, void *ibuf,
              pncx_offset nelems, int itype);

/* ------------------------------------------------------------------------ */
/* Device-resident entry points (new API: the reference has no device side) */
/*   All pointers are device (HBM) pointers except fillp (host).  Calls are  */
/*   asynchronous on `stream` and capture-safe (no allocation, no sync).     */
/*   dstatus: device int; the kernels store NC_ERANGE into it when any       */
/*   element is out of range and never clear it (may be NULL).               */
/* ------------------------------------------------------------------------ */

/* In-place swap of an HBM slab (the config-2 / config-5 hot kernel). */
int pncx_dev_in_swapn(void *dbuf, pncx_offset nelems, int esize,
                      pncx_stream_t stream);

/* Out-of-place swap, dst may equal src (ncx.m4:297-467 swapn2b/4b/8b). */
int pncx_dev_swapn(void *ddst, const void *dsrc, pncx_offset nelems,
                   int esize, pncx_stream_t stream);

int pncx_dev_putn(int cdf_ver, int xtype, void *dxbuf, const void *dibuf,
                  pncx_offset nelems, int itype, const void *fillp,
                  int *dstatus, pncx_stream_t stream);

int pncx_dev_getn(int cdf_ver, int xtype, const void *dxbuf, void *dibuf,
                  pncx_offset nelems, int itype, int *dstatus,
                  pncx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Fill path: fill_var_buf (src/drivers/ncmpio/ncmpio_fill.c:89-140).         */
/* Replicates one external (big-endian) fill value of xtype over nelems      */
/* elements.  xvalue = the _FillValue attribute's external bytes, or NULL    */
/* for the default NC_FILL_<X> pattern (ncmpio_fill.c:50-60).                */
/* ------------------------------------------------------------------------ */
int pncx_dev_fill(int xtype, void *dxbuf, pncx_offset nelems, const void *xvalue,
                  pncx_stream_t stream);
int pncx_fill(int xtype, void *xbuf, pncx_offset nelems, const void *xvalue);

/* ------------------------------------------------------------------------ */
/* varm: internal buffer laid out by imap[] (element strides per dimension,  */
/* ncmpii_create_imaptype, src/drivers/common/create_imaptype.c:25-139),     */
/* external buffer contiguous row-major over count[].  Replaces the MPI_Pack */
/* / MPI_Unpack by the imap type followed by the conversion                 */
/* (ncmpio_util.c:654-689 + 716-765, unpack :842-966) with ONE fused gather  */
/* (put) or scatter (get) kernel.  ndims <= 16; imap[d] >= 0.  For get, the  */
/* imap must not map two packed elements to one user element (the scatter    */
/* order is unspecified, where MPI_Unpack's last-write-wins is not).         */
/* ------------------------------------------------------------------------ */
int pncx_dev_putn_imap(int cdf_ver, int xtype, void *dxbuf, const void *dibuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, int itype,
                       const void *fillp, int *dstatus, pncx_stream_t stream);
int pncx_dev_getn_imap(int cdf_ver, int xtype, const void *dxbuf, void *dibuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, int itype,
                       int *dstatus, pncx_stream_t stream);
/* host buffers: the user-buffer span sum((count-1)*imap)+1 elements is staged */
int pncx_putn_imap(int cdf_ver, int xtype, void *xbuf, const void *ibuf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, int itype, const void *fillp);
int pncx_getn_imap(int cdf_ver, int xtype, const void *xbuf, void *ibuf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, int itype);

/* ------------------------------------------------------------------------ */
/* Derived user-buffer datatypes (the flexible API's bufcount + buftype).    */
/* The reference accepts any MPI derived datatype built from one element     */
/* type as the user-buffer layout (ncmpii_buftype_decode,                    */
/* src/drivers/common/dtype_decode.c:628-694; NC_EMULTITYPES otherwise) and  */
/* packs it with MPI_Pack before converting (ncmpio_pack_xbuf,               */
/* ncmpio_util.c:620-652; MPI_Unpack after converting, :889-933).  Here the  */
/* layout is committed once as its flattened typemap -- nblocks runs of      */
/* blocklen[i] elements of itype at byte displacement disp[i] (any sign), in */
/* pack order, one copy of the typemap every `extent` bytes -- and the       */
/* pack/unpack is fused into the conversion kernel.  include/pncx_ncmpii.h   */
/* flattens an MPI_Datatype into this form (pncx_mpi_type_commit).           */
/* ------------------------------------------------------------------------ */
#ifndef NC_EMULTITYPES
#define NC_EMULTITYPES  (-208)   /* pnetcdf.h.in:629 */
#define NC_EIOMISMATCH  (-209)   /* pnetcdf.h.in:630 */
#endif
typedef struct pncx_dtype pncx_dtype;

/* Validate and normalise (drop empty runs, merge adjacent ones) the typemap,
 * classify it (contiguous / uniform runs / general table) and, for a general
 * table, upload it to HBM once so the device calls below stay asynchronous
 * and capture-safe.  The arrays are copied.  Returns NC_NOERR, NC_EBADTYPE,
 * NC_EINVAL, NC_ENOMEM or PNCX_EDEVICE. */
int pncx_type_commit(int itype, pncx_offset nblocks, const pncx_offset *disp,
                     const pncx_offset *blocklen, pncx_offset extent, pncx_dtype **dtype);
/* Release the caller's reference; pending nonblocking requests keep theirs
 * (MPI_Type_free semantics). */
int pncx_type_free(pncx_dtype *dtype);
/* itype, elements per copy, extent, and layout (0 contiguous, 1 uniform
 * runs, 2 general table) after normalisation; any pointer may be NULL. */
int pncx_type_inq(const pncx_dtype *dtype, int *itype, pncx_offset *nelems, pncx_offset *extent,
                  int *layout);

/* Convert prod(count[0..ndims)) elements (1 when ndims == 0) between the
 * external buffer (contiguous, row-major over count) and a user buffer of
 * `bufcount` copies of `buftype`, with an optional imap[] applied first
 * (packed element index = sum idx_d*imap[d], as the reference packs the
 * buftype and then the imap type, ncmpio_util.c:620-689).  bufcount copies
 * must hold exactly that many elements, else NC_EIOMISMATCH
 * (dtype_decode.c:690).  itype is the buftype's element type.  For get, the
 * typemap must not map two elements to one address (MPI_Unpack into
 * overlapping memory is erroneous).  Other rules as pncx_*_imap. */
int pncx_dev_putn_flex(int cdf_ver, int xtype, void *dxbuf, const void *dbuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                       const pncx_dtype *buftype, const void *fillp, int *dstatus,
                       pncx_stream_t stream);
int pncx_dev_getn_flex(int cdf_ver, int xtype, const void *dxbuf, void *dbuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                       const pncx_dtype *buftype, int *dstatus, pncx_stream_t stream);
/* host buffers: the byte span the bufcount copies cover is staged through HBM
 * (for get it is read first, so bytes between the runs are preserved) */
int pncx_putn_flex(int cdf_ver, int xtype, void *xbuf, const void *buf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                   const pncx_dtype *buftype, const void *fillp);
int pncx_getn_flex(int cdf_ver, int xtype, const void *xbuf, void *buf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                   const pncx_dtype *buftype);

/* MPI_Pack / MPI_Unpack in HBM: bufcount copies of a committed buftype
 * between a user buffer and a contiguous packed buffer of its elements, both
 * on the device, no conversion -- the first step of ncmpio_pack_xbuf
 * (ncmpio_util.c:620-652) and the last of ncmpio_unpack_xbuf (:889-933),
 * used where a packed copy is needed (the flexible varn and bput calls on
 * device buffers).  stream NULL: the call waits for completion. */
int pncx_dev_pack(void *dpacked, const void *dbuf, pncx_offset bufcount, const pncx_dtype *buftype,
                  pncx_stream_t stream);
int pncx_dev_unpack(const void *dpacked, void *dbuf, pncx_offset bufcount, const pncx_dtype *buftype,
                    pncx_stream_t stream);
/* Device memory on the current device (hipMalloc), for such packed copies. */
void *pncx_dev_alloc(pncx_offset nbytes);
int   pncx_dev_free(void *p);

/* ------------------------------------------------------------------------ */
/* Data comparison of ncmpidiff (src/utils/ncmpidiff/ncmpidiff_core.c:200-  */
/* 236, CHECK_VAR_DIFF): the smallest index at which two HBM arrays of      */
/* itype differ -- exactly (tolerance == 0), or (tolerance != 0) when the   */
/* absolute difference exceeds tol_diff AND the ratio to the larger         */
/* magnitude exceeds tol_ratio, with the reference's C arithmetic.          */
/* *first = that index, or -1 when the arrays agree.  Synchronises stream.  */
/* ------------------------------------------------------------------------ */
int pncx_dev_first_diff(const void *da, const void *db, pncx_offset nelems, int itype, int tolerance,
                        double tol_diff, double tol_ratio, pncx_offset *first, pncx_stream_t stream);

/* ------------------------------------------------------------------------ */
/* Batched conversion: many independent requests in one launch per         */
/* conversion class (replaces the per-request loop of                       */
/* ncmpio_igetput_varm, ncmpio_i_getput.m4:300-303, and the per-request      */
/* unpack at wait time, ncmpio_wait.c:743-781).                              */
/* ------------------------------------------------------------------------ */
typedef struct pncx_seg {
    int          dir;       /* PNCX_PUT or PNCX_GET                          */
    int          cdf_ver;   /* 1, 2 or 5                                     */
    int          xtype;     /* NC_BYTE .. NC_UINT64                          */
    int          itype;     /* enum pncx_itype                               */
    pncx_offset  nelems;
    void        *xbuf;      /* external buffer                               */
    void        *ibuf;      /* internal buffer; may equal xbuf for same-type */
    const void  *fillp;     /* PUT only: xtype fill value (native) or NULL   */
} pncx_seg;

/* Device buffers.  status_out[i] (host array, may be NULL) receives the
 * status of segment i after the call completes (this call synchronises the
 * stream).  Returns the first non-NOERR segment status. */
int pncx_dev_batch(const pncx_seg *segs, int nseg, int *status_out,
                   pncx_stream_t stream);

/* Asynchronous form: queues the same launches on `stream` and returns
 * without waiting.  dstatus is a device array of nseg ints that the caller
 * zeroes; segment i's word becomes NC_ERANGE if it had out-of-range values
 * (read it after the stream completes, e.g. pncx_dev_status_read).  The
 * return value reports argument errors (first bad segment) only.  A repeated
 * segment list with the same dstatus reuses the device plan and touches no
 * host staging memory, so calls can be queued back to back; a new plan first
 * waits for the previous async call's stream. */
int pncx_dev_batch_async(const pncx_seg *segs, int nseg, int *dstatus,
                         pncx_stream_t stream);

/* Measurement aid (no reference counterpart): with timing enabled, every
 * pncx_dev_batch and pncx_dev_batch_async call on the current device has
 * its batch kernels stamped with HIP events by their own dispatches (start
 * and end of every class kernel, summed per call; not the descriptor
 * upload, the flag reduce, the status copy or the wait).  A call with more
 * than 256 classes is not timed.  pncx_dev_batch_kernel_ms waits for the
 * calls still queued and returns the summed kernel time and the number of
 * calls timed since pncx_dev_batch_timing(1) (which resets both). */
int pncx_dev_batch_timing(int enable);
int pncx_dev_batch_kernel_ms(double *total_ms, long long *calls);

/* Measurement aid (no reference counterpart): per-phase time of the
 * host-buffer paths (pncx_putn/getn/in_swapn and the file layer's blocking
 * put/get from host buffers).  Off by default, or on from the start with
 * PNCX_PHASES=1 in the environment.  pncx_phases(1) clears the sums and
 * turns recording on, pncx_phases(0) turns it off.  Phase ids run from 0
 * while pncx_phase_name(id) is not NULL; a phase's host time is summed in
 * microseconds with the number of times it ran.  The phases are host
 * clock intervals; with pncx_phases(2) (PNCX_PHASES=2) the first chunks of
 * a staged conversion also get HIP events, summed as "gpu.h2d", "gpu.kernel"
 * and "gpu.d2h" (they serialise the pipeline a little: use them to see
 * the device side, not to time the call). */
int pncx_phases(int enable);
/* A/B switches of the kernel and staging choices (DESIGN.md names each):
 * PNCX_<name> in the environment is read once when the library loads; this
 * changes one for the calls that follow (value -1 restores the default).
 * NC_EINVAL for an unknown name. */
int pncx_knob_set(const char *name, long long value);
int pncx_knob_get(const char *name, long long *value);
const char *pncx_phase_name(int id);
int pncx_phase_read(int id, double *us, long long *count);

/* Host buffers (staged through HBM). */
int pncx_batch(const pncx_seg *segs, int nseg, int *status_out);

/* ------------------------------------------------------------------------ */
/* Runtime helpers                                                           */
/* ------------------------------------------------------------------------ */
int  pncx_device_count(void);
int  pncx_set_device(int dev);
int  pncx_get_device(void);
/* Set up ahead of the first data call on the current device what that call
 * would otherwise pay for: the device context (streams, status words), the
 * staging events and the same-type swap kernels' code object (no reference
 * equivalent; ncmpi_create/ncmpi_open run it on a thread, pncx_nc.c
 * warm_start).  NC_NOERR or PNCX_EDEVICE. */
int  pncx_warmup(void);
/* Load on device `dev` the put and get conversion kernels of the external
 * types in `mask` (bit x = NC type x; NC_CHAR ignored), each type once per
 * device: 9-16 ms per type that the first put or get of the type would pay.
 * ncmpi_enddef runs it on a thread for the types of the defined variables
 * (pncx_nc.c, PNCX_PRELOAD=0 turns that off).  No reference equivalent.
 * NC_NOERR or PNCX_EDEVICE.  pncx_preload_pending: the types of `mask`
 * not loaded on `dev` yet. */
int  pncx_preload_xtypes(int dev, unsigned mask);
unsigned pncx_preload_pending(int dev, unsigned mask);
/* Pin a long-lived host buffer for direct DMA (no reference equivalent: the
 * xbuf of ncmpio_getput.m4:216,422 is malloc'ed per call).  Host entry points
 * pin buffers >= 64 MiB themselves for the duration of a call; a buffer
 * registered here skips that per-call cost (~30 ms per 4 GiB on MI355X
 * hosts).  Returns NC_NOERR, also when the range is already pinned, or
 * PNCX_EDEVICE.  Unregister before freeing the memory. */
int  pncx_host_register(void *buf, pncx_offset nbytes);
int  pncx_host_unregister(void *buf);
/* 1 if p points into device memory (hipMalloc), else 0.  The file layer
 * (pncx_nc.h) and so the ncmpi_* API take such user buffers on the
 * device-resident path: converted in HBM, external bytes across PCIe once. */
int  pncx_is_device_ptr(const void *p);
/* Synchronise `stream` and return *dstatus (NC_NOERR if it was 0). */
int  pncx_dev_status_read(const int *dstatus, pncx_stream_t stream);
const char *pncx_strerror(int err);
/* Version string of the library build (arch, kernel set). */
const char *pncx_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PNCX_H */
