/*
 * pncx_shim.h -- the thin C-ABI between the C host code (pncx_host.c) and
 * the HIP translation units (kernel launchers + HIP runtime wrappers).
 * Internal to libpncx.so; the public boundary is include/pncx.h.
 */
#ifndef PNCX_SHIM_H
#define PNCX_SHIM_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* one streaming launch: n elements from src to dst (may be equal) */
typedef struct pncxk_args {
    const void        *src;
    void              *dst;
    long long          n;
    unsigned long long fill;        /* PUT: native bits of the xtype fill */
    int               *status;      /* device int or NULL                 */
    void              *stream;      /* hipStream_t                        */
    int                nontemporal; /* 1: nt loads/stores                 */
} pncxk_args;

/* one segment of a batched launch (device-resident copy of this array) */
typedef struct pncxk_seg {
    /* what every block of a batch kernel reads first: one 64-byte line */
    const void        *src;
    void              *dst;
    long long          head;   /* scalar elements before the 16B-aligned body */
    long long          nvec;   /* vector steps in the body                    */
    long long          block0; /* first block of this segment                 */
    unsigned long long fill;
    int                aux;    /* SWAPMIX: element size of this segment       */
    int                pad;
    /* the segment's first block (head/remainder) and the flag reduce */
    long long          n;
    int               *status; /* device int of this segment, or NULL         */
} pncxk_seg;

/* up to PNCXK_MAXGRP runs of equal-size segments: block b of the grid is in
 * run k when r[k].b0 <= b < r[k+1].b0, segment r[k].s0 + (b - r[k].b0) / r[k].per.
 * The division is a multiply and a shift: q = (x * mag) >> shr with
 * mag = ceil(2^shr / per), shr = 31 + ceil(log2 per), exact for x < 2^31
 * (a class grid never reaches 2^31 blocks: that would be >= 8 TiB).  One
 * record per run, so a kernel with one or two runs reads 64 contiguous bytes
 * of its arguments (the C4 batches: tools/c4_kernel_ablation.hip). */
#define PNCXK_MAXGRP 8
typedef struct pncxk_run {
    long long          b0;    /* first block of the run            */
    unsigned long long mag;   /* multiplier for / per              */
    long long          per;   /* blocks per segment in this run    */
    int                s0;    /* first segment of the run          */
    int                shr;   /* shift for / per                   */
} pncxk_run;
typedef struct pncxk_groups {
    int       n;
    int       pad;
    pncxk_run r[PNCXK_MAXGRP];
} pncxk_groups;

typedef struct pncxk_batch_args {
    const pncxk_seg *dsegs;    /* device array, sorted by block0           */
    int              nseg;
    long long        nblocks;
    int             *dmap;     /* device block->segment table or NULL      */
    pncxk_groups     grp;      /* block -> segment runs when grp.n > 0, else dmap */
    int              sval;     /* value a segment's status word gets on ERANGE */
    void            *stream;
    void            *ev_start; /* timing events stamped at this launch's start */
    void            *ev_stop;  /* and end (hipExtLaunchKernel), or NULL      */
} pncxk_batch_args;

/* varm layout of the user buffer (create_imaptype.c semantics) */
#define PNCX_MAX_DIMS 16
#define PNCX_TMAP_PIECE 512
typedef struct pncxk_imap {
    int       ndims;
    int       pad;
    long long max_count;
    long long count[PNCX_MAX_DIMS];
    long long imap[PNCX_MAX_DIMS];   /* in elements of the internal type */
    /* flattened user-buffer datatype applied after imap (the MPI_Pack
     * typemap of a derived buftype): the imap offset j is the packed
     * element index; copy c = j / tn sits textent bytes after copy c-1.
     * tmode 0: none, byte offset = j * element size
     *       1: uniform blocks of tlen elements, tstride bytes apart from tdisp0
     *       2: table, tnblk blocks, tpre[b] = first packed element of block b,
     *          tdisp[b] = its byte displacement (device arrays; tpre[tnblk] = tn)
     *       3: the same table, runs long enough for one wave per run (packed
     *          order only; runs split into pieces of <= PNCX_TMAP_PIECE)
     *       4: the same table, short runs: per-element byte map toff
     *       5: the same, 16-bit map: element r at tlo + toff[r >> 6] + toff16[r]
     *       6: the same, 8-bit gap map (toff8, below)
     *       7: the same, 4-bit gap-step map (toff8 holds nibbles, below) */
    int       tmode;
    int       tpad;
    long long tn, textent, tlen, tstride, tdisp0, tnblk;
    const long long *tpre;
    const long long *tdisp;
    const long long *tcidx;          /* tcidx[q]: the block holding element 64q (q <= ceil(tn/64)) */
    /* tmode 4: short-run table with a per-element map: element r of a copy
     * is at byte tlo + toff[r] (device array of tn, built at commit) */
    const unsigned  *toff;
    long long        tlo;
    /* tmode 5: toff holds one base per 64-element chunk, toff16 the offsets
     * from it (2 B per element instead of 4: chunks spanning < 64 KiB) */
    const unsigned short *toff16;
    /* tmode 6: toff holds the byte offset of each chunk's first element, toff8
     * the gap elements before element r in its chunk: r at
     * tlo + toff[r >> 6] + ((r & 63) + toff8[r]) * element size.
     * tmode 7: toff8 holds 32 bytes per chunk (32-byte aligned), one nibble
     * per element (s of chunk q at byte 32q + s/2, low nibble first): the
     * gap elements between element s-1 and s; the gap count before element
     * s is the sum of nibbles 0..s of its chunk */
    const unsigned char *toff8;
} pncxk_imap;

typedef struct pncxk_opinfo {
    int ss;           /* source element bytes       */
    int ds;           /* destination element bytes  */
    int vec;          /* elements per lane per step */
    int batch_steps;  /* steps per lane per block   */
} pncxk_opinfo;

/* operation kinds for batch / opinfo */
#define PNCXK_SWAP 0  /* a = esize (1 = copy)  */
#define PNCXK_GET  1  /* a = xtype, b = itype  */
#define PNCXK_PUT  2  /* a = xtype, b = itype, c = preserve */
#define PNCXK_SWAPMIX 3  /* batch only: same-type swaps/copies of any of 1/2/4/8 bytes */
#define PNCXK_MIX_LANES 1024  /* lanes (x 16 B) per block tile of the SWAPMIX kernel */

/* ---- kernel launchers (HIP TUs) ---- */
int pncxk_swap(int esize, const pncxk_args *a);          /* esize 1,2,4,8 */
int pncxk_swap_generic(int esize, const pncxk_args *a);  /* any esize >= 1 */
int pncxk_get(int xtype, int itype, const pncxk_args *a);
int pncxk_put(int xtype, int itype, int preserve, const pncxk_args *a);
int pncxk_batch(int kind, int a, int b, int c, const pncxk_batch_args *args);
/* one launch for a conversion class (conv) and the same-type swap class
 * (mix) of one batch; PNCXK_NOFUSE when the pair does not fuse (then the
 * caller launches both classes itself) */
#define PNCXK_NOFUSE 1
int pncxk_batch_fused(int kind, int a, int b, int c, const pncxk_batch_args *conv, const pncxk_batch_args *mix);
/* fused varm gather (gather=1: put, src strided) / scatter (get, dst strided) */
int pncxk_launch_imap(int kind, int a, int b, int c, const pncxk_args *args, const pncxk_imap *m, int gather);
int pncxk_opinfo_get(int kind, int a, int b, int c, pncxk_opinfo *o);
/* replicate an xsize-byte external value over nelems elements (device) */
int pncxk_fill(void *dst, long long nelems, int xsize, const void *xvalue, void *stream);
/* smallest index where a and b (n elements of itype) differ, exactly or
 * beyond both tolerances (ncmpidiff); atomicMin into *first (device) */
int pncxk_first_diff(const void *a, const void *b, long long n, int itype, int tol, double td, double tr,
                     unsigned long long *first, void *stream);
/* fill args->dmap (nblocks ints) from the device descriptors */
int pncxk_batch_map(const pncxk_batch_args *args);
/* completion of a synchronous batch: copy n status words to host-mapped
 * hstat, then store seq into host-mapped *hdone (system scope) */
int pncxk_batch_done(const int *dstat, int n, int *hstat, int *hdone, int seq, void *stream);

/* ---- A/B knobs: read from the environment (PNCX_<name>) once when the
 * library loads, changed by pncx_knob_set (include/pncx.h) in tests; -1 =
 * not set, the code's own default applies ---- */
enum {
    PNCXK_KNOB_TILE_U,          /* k_tile_u tiles per block: 1, 2, 4         */
    PNCXK_KNOB_XPOSE_MERGE,     /* 0: transposes tile dimension P alone      */
    PNCXK_KNOB_URUN,            /* 0: uniform runs off k_urun                */
    PNCXK_KNOB_TMAP_VEC,        /* 0: run pieces one element per lane        */
    PNCXK_KNOB_IMAP_ROWS,       /* 0: varm rows off k_imap_rows              */
    PNCXK_KNOB_FUSE_LANES,      /* 1024: fused batch with 1024-lane blocks   */
    PNCXK_KNOB_BATCH_FUSE,      /* 1: fused two-class batch launch           */
    PNCXK_KNOB_TMAP_IMAP,       /* 0: lattice tables stay run pieces         */
    PNCXK_KNOB_TOFF16,          /* 0: 32-bit offset maps                     */
    PNCXK_KNOB_TOFF_MAX_ELEMS,  /* largest short-run table given a map       */
    PNCXK_KNOB_XPOSE_ORDER,     /* transpose tile order (0 row-major)        */
    PNCXK_KNOB_TOFF_RUNS,       /* 0: short-run tables keep the offset map   */
    PNCXK_KNOB_HOST_ZC,         /* host-buffer chunks: 0 copy, 1 zero-copy
                                 * stores, 2 zero-copy both ways, 3 copies on
                                 * alternating streams; unset: by size       */
    PNCXK_KNOB_IO_INLINE_MB,    /* requests below: I/O on the calling thread */
    PNCXK_KNOB_FILE_WINDOW,     /* tmpfs file windows: unset/0 off, 1 at the second touch, 2 at first use */
    PNCXK_KNOB_IO_POPULATE,     /* 0: mapped writes fault their pages in     */
    PNCXK_KNOB_HOST_ZC_MAX_MB,  /* largest call given zero-copy chunks       */
    PNCXK_KNOB_TGAP,            /* 0: 8-bit gap maps stay on k_imap          */
    PNCXK_KNOB_GROW,            /* 0: no fallocate of appended ranges while
                                 * the GPU converts (tmpfs)                  */
    PNCXK_KNOB_READ_SPLIT,      /* pool preads per chunk of an inline get    */
    PNCXK_KNOB_WARM,            /* 0: no device/staging warm-up at create/open */
    PNCXK_KNOB_PRELOAD,         /* 0: no code-object preload of the file's types at enddef */
    PNCXK_KNOB_FAULT,           /* test only: 1 fails an appending put right after its grow */
    PNCXK_NKNOB
};
long long pncx_knob(int id);

/* ---- HIP runtime wrappers (return 0 on success, PNCX_EDEVICE on error) ---- */
int  pncxrt_device_count(void);
int  pncxrt_set_device(int dev);
int  pncxrt_get_device(void);
int  pncxrt_load_swap_code(void);      /* the swap file's code object on the current device */
int  pncxk_load_xtype(int xtype);      /* one external type's put + get code objects (pncx_kern_xt.c) */
int  pncxrt_malloc(void **p, size_t n);
int  pncxrt_free(void *p);
int  pncxrt_host_alloc(void **p, size_t n);
/* fine-grained (coherent) pinned memory the device writes directly: *dp is
 * the device-side address of *p */
int  pncxrt_host_alloc_mapped(void **p, void **dp, size_t n);
int  pncxrt_host_free(void *p);
int  pncxrt_memcpy_h2d(void *d, const void *h, size_t n, void *stream);
int  pncxrt_memcpy_d2h(void *h, const void *d, size_t n, void *stream);
int  pncxrt_memcpy_d2d(void *d, const void *s, size_t n, void *stream);
int  pncxrt_memset(void *d, int v, size_t n, void *stream);
int  pncxrt_stream_create(void **s);
int  pncxrt_stream_destroy(void *s);
int  pncxrt_stream_sync(void *s);
int  pncxrt_event_create(void **e);
int  pncxrt_event_create_fast(void **e);   /* no timing: cheaper record and wait */
int  pncxrt_event_destroy(void *e);
int  pncxrt_event_record(void *e, void *stream);
int  pncxrt_stream_wait_event(void *stream, void *e);
int  pncxrt_event_sync(void *e);
/* 1 = done, 0 = not yet, PNCX_EDEVICE = error */
int  pncxrt_event_query(void *e);
int  pncxrt_event_elapsed_ms(float *ms, void *start, void *stop);
int  pncxrt_is_device_ptr(const void *p);   /* device memory of the current device */
int  pncxrt_ptr_device(const void *p);      /* its device for device memory, else -1 */
/* pin a pageable host range for DMA: 0 = registered by this call (caller
 * unregisters), 1 = already pinned/registered, PNCX_EDEVICE = could not */
int  pncxrt_host_register(void *p, size_t n);
int  pncxrt_host_unregister(void *p);
/* device address of pinned/registered host memory, NULL otherwise */
void *pncxrt_host_dptr(const void *p);
/* the same for a whole range [p, p + n): NULL unless all of it is mapped */
void *pncxrt_host_dptr_range(const void *p, size_t n);
/* register a shared file mapping for device access (read-only or not):
 * 0 = registered, PNCX_EDEVICE = refused */
int  pncxrt_host_register_map(void *p, size_t n, int readonly);
/* host buffers at least this large are pinned for a call (pncx_host.c) */
size_t pncxrt_pin_threshold(void);
const char *pncxrt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
