/*
 * pncx_host.c -- C host side of libpncx: the include/pncx.h entry points.
 *
 * Classifies each request the way the reference's convert_swap.m4 /
 * ncmpio_util.c buffer policy does (copy, byte swap, or cast+swap), builds
 * the launch descriptors, and for host buffers stages the data through HBM
 * in chunks on two HIP streams so the copies of one chunk overlap the
 * kernel of the other.  All device work goes through the thin C-ABI shim
 * (pncx_shim.h); there is no CPU conversion code in this library.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/pncx.h"
#include "pncx_shim.h"
#include "pncx_phase.h"
#include "pncx_stage.h"

/* ------------------------------------------------------------------------ */
/* type metadata                                                             */
/* ------------------------------------------------------------------------ */
int pncx_xlen(int xtype)                     /* ncmpii_xlen_nc_type, utils.c:46-62 */
{
    switch (xtype) {
        case NC_BYTE: case NC_UBYTE: case NC_CHAR: return 1;
        case NC_SHORT: case NC_USHORT: return 2;
        case NC_INT: case NC_UINT: case NC_FLOAT: return 4;
        case NC_DOUBLE: case NC_INT64: case NC_UINT64: return 8;
        default: return -1;
    }
}

int pncx_ilen(int itype)
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

int pncx_need_convert(int format, int xtype, int itype)  /* convert_swap.m4:85-116 */
{
    if (xtype == NC_CHAR) return 0;
    if (format < PNCX_FORMAT_CDF5 && xtype == NC_BYTE && itype == PNCX_ITYPE_UCHAR) return 0;
    if (itype == PNCX_ITYPE_LONG) itype = PNCX_ITYPE_LONGLONG;
    return !((xtype == NC_BYTE   && itype == PNCX_ITYPE_SCHAR)    ||
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

int pncx_need_swap(int xtype, int itype)                 /* common.h:47-54 */
{
    return ((xtype == NC_CHAR  && itype == PNCX_ITYPE_CHAR)  ||
            (xtype == NC_BYTE  && itype == PNCX_ITYPE_SCHAR) ||
            (xtype == NC_UBYTE && itype == PNCX_ITYPE_UCHAR)) ? 0 : 1;
}

const char *pncx_strerror(int err)
{
    switch (err) {
        case NC_NOERR: return "No error";
        case NC_EINVAL: return "Invalid argument";
        case NC_EBADTYPE: return "Not a netcdf data type";
        case NC_ECHAR: return "Attempt to convert between text & numbers";
        case NC_ERANGE: return "Numeric conversion not representable";
        case NC_ENOMEM: return "Memory allocation (malloc) failure";
        case PNCX_EDEVICE: {
            const char *e = pncxrt_last_error();
            return (e && e[0]) ? e : "HIP device error";
        }
        default: return "Unknown error";
    }
}

const char *pncx_version(void) { return "pncx 0.1 gfx950 (swap 2/4/8/n, 10x11 get/put, batch)"; }

/* ------------------------------------------------------------------------ */
/* per-phase timing (pncx_phase.h; pncx_phases in include/pncx.h)            */
/* ------------------------------------------------------------------------ */
int pncx_ph_on;
static double g_ph_us[PH_N];
static long long g_ph_n[PH_N];
static pthread_mutex_t g_ph_lock = PTHREAD_MUTEX_INITIALIZER;
static const char *const g_ph_names[PH_N] = {
    "put.plan", "put.register", "put.convert", "put.write", "put.wait", "put.unregister", "put.total",
    "get.plan", "get.register", "get.read", "get.convert", "get.unregister", "get.total",
    "conv.lock_pin", "conv.enqueue", "conv.sync", "conv.status", "conv.unpin",
    "gpu.h2d", "gpu.kernel", "gpu.d2h", "file.window_map", "file.window_use", "put.grow", "warm", "preload"};

/* A/B knobs (pncx_shim.h): the environment once at load, then pncx_knob_set */
static const char *const g_knob_names[PNCXK_NKNOB] = {
    "TILE_U", "XPOSE_MERGE", "URUN", "TMAP_VEC", "IMAP_ROWS", "FUSE_LANES", "BATCH_FUSE", "TMAP_IMAP",
    "TOFF16", "TOFF_MAX_ELEMS", "XPOSE_ORDER", "TOFF_RUNS", "HOST_ZC", "IO_INLINE_MB", "FILE_WINDOW", "IO_POPULATE", "HOST_ZC_MAX_MB", "TGAP",
    "GROW", "READ_SPLIT", "WARM", "PRELOAD", "FAULT"};
static long long g_knob[PNCXK_NKNOB];

long long pncx_knob(int id)
{
    return id >= 0 && id < PNCXK_NKNOB ? __atomic_load_n(&g_knob[id], __ATOMIC_RELAXED) : -1;
}

static int knob_id(const char *name)
{
    int i;
    if (name == NULL) return -1;
    if (strncmp(name, "PNCX_", 5) == 0) name += 5;
    for (i = 0; i < PNCXK_NKNOB; i++)
        if (strcmp(name, g_knob_names[i]) == 0) return i;
    return -1;
}

int pncx_knob_set(const char *name, long long value)
{
    const int id = knob_id(name);
    if (id < 0) return NC_EINVAL;
    __atomic_store_n(&g_knob[id], value < 0 ? -1 : value, __ATOMIC_RELAXED);
    return NC_NOERR;
}

int pncx_knob_get(const char *name, long long *value)
{
    const int id = knob_id(name);
    if (id < 0) return NC_EINVAL;
    if (value) *value = pncx_knob(id);
    return NC_NOERR;
}

static int g_nontemporal;
static size_t g_chunk_bytes, g_pin_min;

/* The environment, read once at load, before any thread of the library
 * runs (no lazily set globals that two threads could race on): phases,
 * the A/B knobs and the size settings below. */
__attribute__((constructor)) static void ph_init(void)
{
    const char *e;
    char nm[64];
    int i;
    long v;
    e = getenv("PNCX_NONTEMPORAL");              /* -1: plain accesses (A/B) */
    g_nontemporal = e ? atoi(e) : 1;
    e = getenv("PNCX_CHUNK_MB");
    v = e ? atol(e) : 16;
    g_chunk_bytes = (size_t)(v > 0 ? v : 16) << 20;
    e = getenv("PNCX_PIN_MIN_KB");
    v = e ? atol(e) : 1024;
    g_pin_min = (size_t)(v > 0 ? v : 1024) << 10;
    e = getenv("PNCX_PHASES");
    pncx_ph_on = e != NULL ? (atoi(e) < 0 ? 0 : atoi(e) > 2 ? 2 : atoi(e)) : 0;
    for (i = 0; i < PNCXK_NKNOB; i++) {
        snprintf(nm, sizeof nm, "PNCX_%s", g_knob_names[i]);
        e = getenv(nm);
        g_knob[i] = (e != NULL && e[0] != '\0') ? atoll(e) : -1;
        if (g_knob[i] < -1) g_knob[i] = -1;
    }
}

double pncx_ph_now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}

void pncx_ph_add_us(int id, double us)
{
    if (id < 0 || id >= PH_N) return;
    pthread_mutex_lock(&g_ph_lock);
    g_ph_us[id] += us;
    g_ph_n[id]++;
    pthread_mutex_unlock(&g_ph_lock);
}

int pncx_phases(int enable)
{
    pthread_mutex_lock(&g_ph_lock);
    if (enable) {
        memset(g_ph_us, 0, sizeof g_ph_us);
        memset(g_ph_n, 0, sizeof g_ph_n);
    }
    pncx_ph_on = enable < 0 ? 0 : enable > 2 ? 2 : enable;
    pthread_mutex_unlock(&g_ph_lock);
    return NC_NOERR;
}

const char *pncx_phase_name(int id) { return id >= 0 && id < PH_N ? g_ph_names[id] : NULL; }

int pncx_phase_read(int id, double *us, long long *count)
{
    if (id < 0 || id >= PH_N) return NC_EINVAL;
    pthread_mutex_lock(&g_ph_lock);
    if (us) *us = g_ph_us[id];
    if (count) *count = g_ph_n[id];
    pthread_mutex_unlock(&g_ph_lock);
    return NC_NOERR;
}

int pncx_device_count(void) { return pncxrt_device_count(); }
int pncx_set_device(int dev) { return pncxrt_set_device(dev); }
int pncx_get_device(void) { return pncxrt_get_device(); }

int pncx_is_device_ptr(const void *p)
{
    return p != NULL && pncxrt_is_device_ptr(p);
}

int pncx_host_register(void *buf, pncx_offset nbytes)
{
    if (buf == NULL || nbytes <= 0) return NC_EINVAL;
    if (pncxrt_device_count() <= 0) return PNCX_EDEVICE;
    return pncxrt_host_register(buf, (size_t)nbytes) >= 0 ? NC_NOERR : PNCX_EDEVICE;
}

int pncx_host_unregister(void *buf)
{
    if (buf == NULL) return NC_EINVAL;
    if (pncxrt_device_count() <= 0) return PNCX_EDEVICE;
    return pncxrt_host_unregister(buf) == 0 ? NC_NOERR : PNCX_EDEVICE;
}

/* ------------------------------------------------------------------------ */
/* classification of one request                                             */
/* ------------------------------------------------------------------------ */
typedef struct op_t {
    int kind;      /* PNCXK_SWAP / PNCXK_GET / PNCXK_PUT       */
    int a, b, c;   /* esize | xtype, itype, preserve          */
    int ss, ds;    /* source / destination element bytes      */
    unsigned long long fill;
} op_t;

static int null_fill_preserves(int xtype, int itype)
{
    return xtype == NC_BYTE || xtype == NC_UBYTE ||
           ((xtype == NC_USHORT || xtype == NC_UINT) && itype == PNCX_ITYPE_SCHAR);
}

static unsigned long long default_fill_bits(int xtype)   /* pnetcdf.h.in:104-114 */
{
    unsigned long long b = 0;
    switch (xtype) {
        case NC_BYTE:   { signed char v = PNCX_FILL_BYTE; memcpy(&b, &v, 1); break; }
        case NC_UBYTE:  { unsigned char v = PNCX_FILL_UBYTE; memcpy(&b, &v, 1); break; }
        case NC_SHORT:  { short v = PNCX_FILL_SHORT; memcpy(&b, &v, 2); break; }
        case NC_USHORT: { unsigned short v = PNCX_FILL_USHORT; memcpy(&b, &v, 2); break; }
        case NC_INT:    { int v = PNCX_FILL_INT; memcpy(&b, &v, 4); break; }
        case NC_UINT:   { unsigned v = PNCX_FILL_UINT; memcpy(&b, &v, 4); break; }
        case NC_FLOAT:  { float v = PNCX_FILL_FLOAT; memcpy(&b, &v, 4); break; }
        case NC_DOUBLE: { double v = PNCX_FILL_DOUBLE; memcpy(&b, &v, 8); break; }
        case NC_INT64:  { long long v = PNCX_FILL_INT64; memcpy(&b, &v, 8); break; }
        case NC_UINT64: { unsigned long long v = PNCX_FILL_UINT64; memcpy(&b, &v, 8); break; }
        default: break;
    }
    return b;
}

/* dir: PNCX_PUT or PNCX_GET.  Mirrors ncmpii_{put,get}n_NC_<X> dispatch
 * (convert_swap.m4:202-330) including the CDF-1/2 NC_BYTE<->uchar copy. */
static int classify(int dir, int cdf_ver, int xtype, int itype, const void *fillp, op_t *op)
{
    const int xs = pncx_xlen(xtype), is = pncx_ilen(itype);
    memset(op, 0, sizeof *op);
    if (xs < 0 || is < 0) return NC_EBADTYPE;
    if ((xtype == NC_CHAR) != (itype == PNCX_ITYPE_CHAR)) return NC_ECHAR;
    if (dir != PNCX_PUT && dir != PNCX_GET) return NC_EINVAL;
    op->ss = dir == PNCX_PUT ? is : xs;
    op->ds = dir == PNCX_PUT ? xs : is;
    if (xtype == NC_CHAR || !pncx_need_convert(cdf_ver, xtype, itype)) {
        op->kind = PNCXK_SWAP;        /* same representation: swap (or copy) */
        op->a = xs;
        return NC_NOERR;
    }
    op->kind = dir == PNCX_PUT ? PNCXK_PUT : PNCXK_GET;
    op->a = xtype;
    op->b = itype;
    if (dir == PNCX_PUT) {
        if (fillp != NULL) memcpy(&op->fill, fillp, (size_t)xs);
        else {
            op->fill = default_fill_bits(xtype);
            op->c = null_fill_preserves(xtype, itype);
        }
    }
    return NC_NOERR;
}

/* nontemporal ("streaming") loads/stores: on by default (every byte is
 * touched once); PNCX_NONTEMPORAL=-1 selects plain accesses for A/B runs. */
static int nontemporal_mode(void) { return g_nontemporal; }

static int launch_op(const op_t *op, const void *src, void *dst, long long n, int *dstatus,
                     void *stream)
{
    pncxk_args a;
    a.src = src;
    a.dst = dst;
    a.n = n;
    a.fill = op->fill;
    a.status = dstatus;
    a.stream = stream;
    a.nontemporal = nontemporal_mode();
    switch (op->kind) {
        case PNCXK_SWAP: return pncxk_swap(op->a, &a);
        case PNCXK_GET: return pncxk_get(op->a, op->b, &a);
        case PNCXK_PUT: return pncxk_put(op->a, op->b, op->c, &a);
        default: return NC_EINVAL;
    }
}

/* a device count above zero stays so for the process: cached, so that every
 * call does not ask the runtime again */
static int g_have_dev;
static int have_device(void)
{
    if (__atomic_load_n(&g_have_dev, __ATOMIC_RELAXED)) return 1;
    if (pncxrt_device_count() <= 0) return 0;
    __atomic_store_n(&g_have_dev, 1, __ATOMIC_RELAXED);
    return 1;
}

/* ------------------------------------------------------------------------ */
/* device-resident entry points                                              */
/* ------------------------------------------------------------------------ */
int pncx_dev_swapn(void *ddst, const void *dsrc, pncx_offset nelems, int esize,
                   pncx_stream_t stream)
{
    pncxk_args a;
    if (esize <= 0) return NC_EINVAL;
    if (nelems <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    if (esize == 1 && ddst == dsrc) return NC_NOERR;
    memset(&a, 0, sizeof a);
    a.src = dsrc;
    a.dst = ddst;
    a.n = nelems;
    a.stream = stream;
    a.nontemporal = nontemporal_mode();
    return pncxk_swap(esize, &a);
}

int pncx_dev_in_swapn(void *dbuf, pncx_offset nelems, int esize, pncx_stream_t stream)
{
    if (esize <= 1 || nelems <= 0) return NC_NOERR;          /* convert_swap.m4:147 */
    return pncx_dev_swapn(dbuf, dbuf, nelems, esize, stream);
}

int pncx_dev_putn(int cdf_ver, int xtype, void *dxbuf, const void *dibuf, pncx_offset nelems,
                  int itype, const void *fillp, int *dstatus, pncx_stream_t stream)
{
    op_t op;
    int err = classify(PNCX_PUT, cdf_ver, xtype, itype, fillp, &op);
    if (err != NC_NOERR) return err;
    if (nelems <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    if (op.kind == PNCXK_SWAP && op.a == 1 && dxbuf == dibuf) return NC_NOERR;
    return launch_op(&op, dibuf, dxbuf, nelems, dstatus, stream);
}

int pncx_dev_getn(int cdf_ver, int xtype, const void *dxbuf, void *dibuf, pncx_offset nelems,
                  int itype, int *dstatus, pncx_stream_t stream)
{
    op_t op;
    int err = classify(PNCX_GET, cdf_ver, xtype, itype, NULL, &op);
    if (err != NC_NOERR) return err;
    if (nelems <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    if (op.kind == PNCXK_SWAP && op.a == 1 && dxbuf == dibuf) return NC_NOERR;
    return launch_op(&op, dxbuf, dibuf, nelems, dstatus, stream);
}

int pncx_dev_status_read(const int *dstatus, pncx_stream_t stream)
{
    int v = 0, err;
    if (dstatus == NULL) return NC_NOERR;
    err = pncxrt_memcpy_d2h(&v, dstatus, sizeof v, stream);
    if (err == 0) err = pncxrt_stream_sync(stream);
    if (err != 0) return PNCX_EDEVICE;
    return v;
}

/* ------------------------------------------------------------------------ */
/* per-device staging context for host-buffer calls                          */
/* ------------------------------------------------------------------------ */
#define NSLOT 2
#define MAX_DEV 64

#define NTEV 256              /* event pairs of pncx_dev_batch_timing read in one go */
#define PH_EVCH 8             /* chunks per call given phase events */
typedef struct ctx_t {
    int    init;
    void  *stream[NSLOT];
    void  *dbuf[NSLOT];       /* device staging, one per slot  */
    size_t dbuf_size;
    int   *dstatus;           /* device status words [NSLOT]   */
    void  *dscratch;          /* batch descriptors / statuses  */
    size_t dscratch_size;
    void  *hscratch;          /* pinned host mirror of dscratch */
    size_t hscratch_size;
    pthread_mutex_t lock;
    void  *barena;            /* device arena of pncx_batch, kept across calls */
    size_t barena_size;
    pthread_mutex_t block;
    /* pncx_dev_batch: the last plan, reused when the same segment list comes
     * again (descriptors still on the device; statuses carry a per-call
     * epoch value, so they need no zeroing) */
    int    epoch;
    int    cache_valid, cache_nseg, cache_ncls;
    int    cache_swaponly;    /* cached plan holds only swaps/copies: no statuses to read */
    int   *cache_dstatus;     /* statuses of the cached plan: NULL = dscratch (synchronous
                               * pncx_dev_batch), else the caller's (pncx_dev_batch_async) */
    void  *async_stream;      /* stream of the last async upload not yet known complete */
    int    async_pending;
    struct pncx_seg *cache_segs;
    uint64_t *cache_fills;    /* the bytes *fillp held when the plan was made: the
                               * plan carries the fill value (classify), the
                               * segment array only its address */
    struct cls_t *cache_cls;
    size_t cache_soff, cache_moff;
    int   *hdone_h, *hdone_d; /* host-mapped completion word [0] + statuses [16..]
                               * of the synchronous pncx_dev_batch (host / device address) */
    int    hdone_cap;         /* status words it holds */
    int    done_seq;
    int    timing;            /* pncx_dev_batch_timing: events around the batch kernels */
    void  *tev[2 * NTEV];     /* start/stop event pairs of the timed calls not yet read */
    int    tpend;             /* pairs in use */
    int    tcpend;            /* timed calls whose pairs are not read yet */
    int    tnext;             /* pairs the call being launched uses      */
    double tms;               /* summed kernel time of the timed batch calls */
    long long tcalls;         /* ... and their number                         */
    unsigned long long *dfirst;   /* pncx_dev_first_diff result word */
    void  *pev[4 * PH_EVCH];  /* pncx_phases: H2D / kernel / D2H events of the first chunks */
    /* staged host-buffer calls (pncx_stage_*): a ring of device slots, an
     * event per chunk after its kernel and after its D2H, a pinned status word */
    void  *sdbuf[4];
    size_t sdbuf_size;
    void  *sev_conv[32], *sev_out[32], *sev_init;
    int   *hstat;
} ctx_t;

static ctx_t g_ctx[MAX_DEV];
static pthread_mutex_t g_ctx_lock = PTHREAD_MUTEX_INITIALIZER;

static size_t chunk_bytes(void) { return g_chunk_bytes; }

static ctx_t *get_ctx(void)
{
    int dev = pncxrt_get_device(), i;
    ctx_t *c;
    if (dev < 0 || dev >= MAX_DEV) return NULL;
    c = &g_ctx[dev];
    pthread_mutex_lock(&g_ctx_lock);
    if (!c->init) {
        int err = 0;
        memset(c, 0, sizeof *c);
        pthread_mutex_init(&c->lock, NULL);
        pthread_mutex_init(&c->block, NULL);
        for (i = 0; i < NSLOT && !err; i++) err = pncxrt_stream_create(&c->stream[i]);
        if (!err) err = pncxrt_malloc((void **)&c->dstatus, NSLOT * sizeof(int));
        if (err) {
            pthread_mutex_unlock(&g_ctx_lock);
            return NULL;
        }
        c->init = 1;
    }
    pthread_mutex_unlock(&g_ctx_lock);
    return c;
}

static int ensure_dbuf(ctx_t *c, size_t need)
{
    int i;
    if (c->dbuf_size >= need) return 0;
    for (i = 0; i < NSLOT; i++) {
        if (c->stream[i]) pncxrt_stream_sync(c->stream[i]);
        pncxrt_free(c->dbuf[i]);
        c->dbuf[i] = NULL;
    }
    c->dbuf_size = 0;
    for (i = 0; i < NSLOT; i++)
        if (pncxrt_malloc(&c->dbuf[i], need) != 0) return PNCX_EDEVICE;
    c->dbuf_size = need;
    return 0;
}

static int ensure_scratch(ctx_t *c, size_t need)
{
    if (c->dscratch_size >= need && c->hscratch_size >= need) return 0;
    need = need < 65536 ? 65536 : need * 2;
    c->cache_valid = 0;                /* the cached descriptors live in dscratch */
    pncxrt_stream_sync(c->stream[0]);
    pncxrt_free(c->dscratch);
    pncxrt_host_free(c->hscratch);
    c->dscratch = c->hscratch = NULL;
    c->dscratch_size = c->hscratch_size = 0;
    if (pncxrt_malloc(&c->dscratch, need) != 0) return PNCX_EDEVICE;
    if (pncxrt_host_alloc(&c->hscratch, need) != 0) return PNCX_EDEVICE;
    c->dscratch_size = c->hscratch_size = need;
    return 0;
}

#define ALIGN16(x) (((x) + 15) & ~(size_t)15)

/*
 * Large host buffers are pinned for the duration of the call
 * (hipHostRegister: ~8 ms for 4 GiB on the MI355X host) so the chunk copies
 * are true async DMA; measured 43 GiB/s of slab for the 8-byte swap vs 26
 * from pageable memory (tools/pcie_probe.py).  Buffers that
 * are already pinned are used as they are; if pinning fails the pageable
 * path is used.
 */
/* smallest host buffer pinned for a call (PNCX_PIN_MIN_KB, default 1 MiB:
 * the file-level sweep of 256 KiB / 1 MiB / 64 MiB, profiles/r01_file_bench_pin*.json) */
size_t pncxrt_pin_threshold(void) { return g_pin_min; }

typedef struct pinned_t { void *p[2]; int n; } pinned_t;

static void pin_range(pinned_t *pn, const void *p, size_t bytes)
{
    int i;
    if (bytes < pncxrt_pin_threshold() || p == NULL) return;
    for (i = 0; i < pn->n; i++)
        if (pn->p[i] == p) return;
    if (pncxrt_host_register((void *)p, bytes) == 0) pn->p[pn->n++] = (void *)p;
}

static void unpin_all(pinned_t *pn)
{
    int i;
    for (i = 0; i < pn->n; i++) pncxrt_host_unregister(pn->p[i]);
    pn->n = 0;
}

/*
 * Staged conversion of host buffers through HBM (pncx_stage.h).
 *
 * A call is cut into chunks.  Each chunk's input is copied to a device slot
 * and converted on the "in" stream; its result is copied back on the "out"
 * stream once the kernel's event has fired.  With the two copy directions
 * on different streams, chunk k+1's H2D overlaps chunk k's D2H (PCIe is
 * full duplex): a 4 MiB swap moves in ~1.3x one direction's copy time
 * instead of 2x (tools/c1_probe.hip, profiles/r04a_c1_probe_4m.txt).  The
 * caller can wait for chunk k alone (pncx_stage_wait) and hand it to file
 * I/O while later chunks are still converting -- the file layer's put/get
 * pipelines (pncx_nc.c).  The ring of NDBUF device slots is reused in
 * order: chunk k's H2D waits for chunk k-NDBUF's D2H on the device.
 *
 * preserve: the destination's current content is needed (NULL-fill codecs).
 */
#define NDBUF 4
#define NSEV 32                     /* chunks in flight (event ring)       */
/* How a chunk crosses PCIe (PNCX_HOST_ZC knob; tools/c1_probe.hip on MI355X,
 * 4 MiB 4-byte swap, profiles/r04d_c1_probe_4m.txt):
 *   STAGE_COPY  H2D (SDMA), kernel in HBM, D2H (SDMA)        1 chunk 185 us
 *   STAGE_ZCOUT H2D (SDMA), kernel stores to the host        4 chunks: 68 us to
 *               destination directly (zero-copy stores)      the first, 178 all
 *   STAGE_ZC    the kernel loads from and stores to host     2 chunks 149 us
 *               memory (no SDMA)
 *   STAGE_ALT   as STAGE_COPY, each chunk wholly on one of two streams,
 *               alternating (round 3's staging)
 * The zero-copy modes need a host destination (and for STAGE_ZC a source)
 * that is pinned or registered; otherwise the chunk takes the next mode
 * down.  STAGE_ZC is the default: 2 GiB in-place 8-byte swap 29-31 GiB/s
 * of slab against 26-27 for the others; NC_INT -> double 61 GiB/s moved
 * against 45 for STAGE_COPY; 1 GiB file gets 28-32 GiB/s against 21-25
 * (profiles/r04j_host_modes.txt). */
enum { STAGE_COPY = 0, STAGE_ZCOUT = 1, STAGE_ZC = 2, STAGE_ALT = 3 };

struct pncx_stage {
    ctx_t *c;
    op_t op;
    int mode;
    int preserve, want_status;
    long long chunk;                /* elements per device slot            */
    size_t din_bytes;               /* input part of a slot                */
    int pushed, waited;             /* chunks enqueued / known complete    */
    int err;
    pinned_t pn;
    int ph_ev;
    /* device-accessible host ranges resolved once per call (pncx_stage_hint):
     * a push inside one of them needs no runtime lookup (two pointer-attribute
     * and two device-pointer queries per side and chunk otherwise, 40-50 us
     * per 4-chunk call on some hosts) */
    struct { const char *h; size_t n; char *d; } hint[4];
    int nhint;
};

/* device address of host range [p, p + n), from the call's hints or the runtime */
static void *stage_dptr(pncx_stage *h, const void *p, size_t n)
{
    int i;
    for (i = 0; i < h->nhint; i++)
        if ((const char *)p >= h->hint[i].h && (const char *)p + n <= h->hint[i].h + h->hint[i].n)
            return h->hint[i].d + ((const char *)p - h->hint[i].h);
    return pncxrt_host_dptr_range(p, n);
}

/* the caller's whole host buffer (or staging area), resolved once */
void pncx_stage_hint(pncx_stage *h, const void *p, size_t n)
{
    char *d;
    if (h == NULL || p == NULL || n == 0 || h->nhint >= 4) return;
    if ((d = (char *)pncxrt_host_dptr_range(p, n)) == NULL) return;
    h->hint[h->nhint].h = (const char *)p;
    h->hint[h->nhint].n = n;
    h->hint[h->nhint].d = d;
    h->nhint++;
}

static int stage_slots(ctx_t *c, size_t slot_bytes)
{
    int i;
    if (c->sev_init == NULL) {
        for (i = 0; i < NSEV; i++)
            if (pncxrt_event_create_fast(&c->sev_conv[i]) || pncxrt_event_create_fast(&c->sev_out[i]))
                return PNCX_EDEVICE;
        if (pncxrt_event_create_fast(&c->sev_init)) return PNCX_EDEVICE;
    }
    if (c->hstat == NULL && pncxrt_host_alloc((void **)&c->hstat, 64) != 0) return PNCX_EDEVICE;
    if (c->sdbuf_size >= slot_bytes || slot_bytes == 0) return 0;
    for (i = 0; i < NSLOT; i++) pncxrt_stream_sync(c->stream[i]);
    for (i = 0; i < NDBUF; i++) {
        pncxrt_free(c->sdbuf[i]);
        c->sdbuf[i] = NULL;
    }
    c->sdbuf_size = 0;
    for (i = 0; i < NDBUF; i++)
        if (pncxrt_malloc(&c->sdbuf[i], slot_bytes) != 0) return PNCX_EDEVICE;
    c->sdbuf_size = slot_bytes;
    return 0;
}

/* What the first staged call on this device would set up: the context
 * (streams, status words), the chunk events, the pinned status word and the
 * swap kernels' code object (4-5 ms).  The file layer runs it on a thread at
 * create/open (pncx_nc.c, warm_start).  The per-type conversion objects stay
 * lazy: loading every kernel file up front made create..enddef 330-530 ms
 * (profiles/r05l_first_call_all_code_objects.txt), and a process converts
 * few external types. */
/* device slots made at warm-up: a 4 MiB record in 1 MiB chunks needs 2-3
 * MiB a slot (C1, C3's reads); larger chunks regrow them at first use */
#define WARM_SLOT_BYTES (16u << 20)
int pncx_warmup(void)
{
    ctx_t *c;
    int err;
    if (!have_device() || (c = get_ctx()) == NULL) return PNCX_EDEVICE;
    pthread_mutex_lock(&c->lock);
    err = stage_slots(c, 0);
    /* Since the staging moves host buffers with the copy engines (round 6,
     * stage_mode), a process's first staged call also paid for the slots'
     * hipMalloc and the first copy on each stream: the first 4 MiB put of
     * the C1 pattern took 18 ms against 1.3 with zero copy
     * (profiles/r06v_c1_first_put.txt).  Both are done here, at enddef. */
    if (!err) err = stage_slots(c, WARM_SLOT_BYTES);
    if (!err) err = pncxrt_memcpy_h2d(c->sdbuf[0], c->hstat, 64, c->stream[0]);
    if (!err) err = pncxrt_memcpy_d2h(c->hstat, c->sdbuf[1], 64, c->stream[1]);
    if (!err) {
        /* and copies from and to memory registered for a call, as the user's
         * buffers are (the first such copy cost ~16 ms more than one from
         * pinned memory) */
        const size_t wb = 1u << 20;
        void *w = aligned_alloc(4096, wb);
        if (w != NULL) {
            memset(w, 0, wb);
            if (pncxrt_host_register(w, wb) == 0) {
                err = pncxrt_memcpy_h2d(c->sdbuf[0], w, wb, c->stream[0]);
                if (!err) err = pncxrt_memcpy_d2h(w, c->sdbuf[1], wb, c->stream[1]);
                if (!err) err = pncxrt_stream_sync(c->stream[0]);
                if (!err) err = pncxrt_stream_sync(c->stream[1]);
                pncxrt_host_unregister(w);
            }
            free(w);
        }
    }
    if (!err) err = pncxrt_stream_sync(c->stream[0]);
    if (!err) err = pncxrt_stream_sync(c->stream[1]);
    pthread_mutex_unlock(&c->lock);
    if (!err && pncxrt_load_swap_code() != 0) err = PNCX_EDEVICE;
    return err;
}

/* The put and get code objects of the external types in `mask` (bit x =
 * NC type x) on device `dev`, each loaded once per device: 9-16 ms apiece,
 * which the first put or get of a new type paid inside the call
 * (profiles/r05p_first_call.txt).  The file layer runs this on a thread at
 * enddef, where the defined variables' types are known (pncx_nc.c). */
static unsigned g_loaded_xt[MAX_DEV];
static pthread_mutex_t g_load_lock = PTHREAD_MUTEX_INITIALIZER;
int pncx_preload_xtypes(int dev, unsigned mask)
{
    int x, err = 0;
    if (dev < 0 || dev >= MAX_DEV || !have_device() || pncxrt_set_device(dev) != 0) return PNCX_EDEVICE;
    for (x = 1; x < 32 && !err; x++) {
        unsigned have;
        if (!(mask & (1u << x)) || x == NC_CHAR) continue;
        pthread_mutex_lock(&g_load_lock);
        have = g_loaded_xt[dev];
        pthread_mutex_unlock(&g_load_lock);
        if (have & (1u << x)) continue;
        err = pncxk_load_xtype(x);
        if (err == NC_EBADTYPE) { err = 0; continue; }
        pthread_mutex_lock(&g_load_lock);
        if (!err) g_loaded_xt[dev] |= 1u << x;
        pthread_mutex_unlock(&g_load_lock);
    }
    return err;
}

/* the types of `mask` not yet loaded on device `dev` */
unsigned pncx_preload_pending(int dev, unsigned mask)
{
    unsigned have;
    if (dev < 0 || dev >= MAX_DEV) return 0;
    pthread_mutex_lock(&g_load_lock);
    have = g_loaded_xt[dev];
    pthread_mutex_unlock(&g_load_lock);
    return mask & ~have & ~(1u << NC_CHAR);
}

/* elements per chunk for a call of n elements: about 4 chunks, each of
 * 1 MiB of input + output at least, chunk_bytes() at most */
static long long stage_chunk_elems(const op_t *op, long long n)
{
    const long long per = op->ss + op->ds;
    long long lo = (1LL << 20) / per, hi = (long long)chunk_bytes() / per, c = (n + 3) / 4;
    if (lo < 1) lo = 1;
    if (hi < lo) hi = lo;
    if (c < lo) c = lo;
    if (c > hi) c = hi;
    return c < n ? c : (n > 0 ? n : 1);
}

/* Chunk mode of a call moving `bytes` (input + output): PNCX_HOST_ZC, else
 * zero copy both ways, up to PNCX_HOST_ZC_MAX_MB when that is set (SDMA
 * copies on alternating streams above it).  Zero copy won at every size
 * measured: 2 GiB round trips 29-31 GiB/s against 27 (alternating copies) and
 * 25 (copy in / copy out streams); file_bench's big get 32.6 against 22.8
 * GiB/s, C3 22.3 against 16.4, C4 16.3 against 12.0
 * (profiles/r04q_host_modes.txt) */
/*
 * Round 6: SDMA copies are the default.  The file-layer fuzz
 * (tests/test_gpu_file_fuzz.py) and tools/window_probe.py found files and
 * user buffers holding stale 64-byte pieces after host-buffer puts and gets
 * whose kernels loaded from or stored to the user's buffer directly (zero
 * copy through the registration made for the call): 9-10 of 150 probe
 * rounds with STAGE_ZC, gets still wrong with STAGE_ZCOUT (the kernel
 * storing into the user buffer), none with STAGE_COPY, where only the copy
 * engines touch the user's pages (profiles/r06u_window_probe.txt).  Direct
 * probes of kernel loads and stores on pinned and registered memory
 * (tools/coherence_probe.hip, tools/visibility_probe.hip,
 * tools/thp_register_probe.py) did not reproduce it, so the cause is not
 * pinned down; the zero-copy modes stay for A/B (PNCX_HOST_ZC=1/2).
 */
static int stage_mode(long long bytes)
{
    const long long m = pncx_knob(PNCXK_KNOB_HOST_ZC), mx = pncx_knob(PNCXK_KNOB_HOST_ZC_MAX_MB);
    if (m >= 0) return m > STAGE_ALT ? STAGE_COPY : (int)m;
    return mx < 0 || bytes <= mx * (1LL << 20) ? STAGE_COPY : STAGE_ALT;
}

static int stage_open(pncx_stage **hp, const op_t *op, int preserve, long long max_chunk, long long total)
{
    pncx_stage *h;
    ctx_t *c = get_ctx();
    int err;
    double t0 = PH_T0();
    *hp = NULL;
    if (c == NULL) return PNCX_EDEVICE;
    if ((h = (pncx_stage *)calloc(1, sizeof *h)) == NULL) return NC_ENOMEM;
    h->c = c;
    h->op = *op;
    h->preserve = preserve;
    /* a same-type swap cannot report NC_ERANGE: no status word to zero or read */
    h->want_status = op->kind != PNCXK_SWAP;
    h->chunk = max_chunk > 0 ? max_chunk : 1;
    h->din_bytes = ALIGN16((size_t)h->chunk * (size_t)op->ss);
    h->mode = stage_mode(total * (long long)(op->ss + op->ds));
    pthread_mutex_lock(&c->lock);
    err = stage_slots(c, h->din_bytes + ALIGN16((size_t)h->chunk * (size_t)op->ds));
    if (!err && h->want_status) {
        /* both streams' kernels may set the word: zero it before either runs */
        err = pncxrt_memset(c->dstatus, 0, sizeof(int), c->stream[0]);
        if (!err) err = pncxrt_event_record(c->sev_init, c->stream[0]);
        if (!err) err = pncxrt_stream_wait_event(c->stream[1], c->sev_init);
    }
    if (!err && pncx_ph_on && c->pev[0] == NULL) {
        int i;
        for (i = 0; i < 4 * PH_EVCH; i++)
            if (pncxrt_event_create(&c->pev[i]) != 0) { c->pev[i] = NULL; break; }
    }
    PH_ADD(PH_CONV_LOCK, t0);
    if (err) {
        pthread_mutex_unlock(&c->lock);
        free(h);
        return err;
    }
    *hp = h;
    return NC_NOERR;
}

int pncx_stage_begin(pncx_stage **hp, int dir, int cdf_ver, int xtype, int itype, const void *fillp,
                     long long max_chunk, long long total)
{
    op_t op;
    int err;
    if (hp) *hp = NULL;
    if (hp == NULL) return NC_EINVAL;
    if (dir == PNCX_SWAP_DIR) {
        memset(&op, 0, sizeof op);
        op.kind = PNCXK_SWAP;
        op.a = op.ss = op.ds = xtype;           /* xtype carries the element size */
        if (xtype < 1) return NC_EINVAL;
    } else if ((err = classify(dir, cdf_ver, xtype, itype, fillp, &op)) != NC_NOERR) {
        return err;
    }
    if (!have_device()) return PNCX_EDEVICE;
    return stage_open(hp, &op, dir == PNCX_PUT ? op.c : 0, max_chunk, total);
}

/* enqueue n (<= the handle's chunk) elements src -> dst; returns the chunk
 * index (>= 0) or an error (< 0) */
int pncx_stage_push(pncx_stage *h, const void *src, void *dst, long long n)
{
    ctx_t *c = h->c;
    const op_t *op = &h->op;
    const int k = h->pushed, slot = k % NDBUF, e = k % NSEV;
    uint8_t *din = (uint8_t *)c->sdbuf[slot], *dout = din + h->din_bytes;
    void *si = c->stream[0], *so = c->stream[1];
    void **ev = NULL;
    int err = h->err;
    double t0 = PH_T0();
    if (err) return err;
    if (n <= 0 || n > h->chunk) return NC_EINVAL;
    if (k - h->waited >= NSEV) {                   /* the event ring is full: wait the oldest */
        if ((err = pncx_stage_wait(h, k - NSEV)) != NC_NOERR) return err;
    }
    if (pncx_ph_on > 1 && c->pev[4 * PH_EVCH - 1] && h->ph_ev < PH_EVCH) ev = &c->pev[4 * h->ph_ev++];
    if ((h->mode == STAGE_ZCOUT || h->mode == STAGE_ZC) && !(op->kind == PNCXK_SWAP && op->a == 1)) {
        /* zero-copy: the kernel writes the host destination itself */
        void *ddst = stage_dptr(h, dst, (size_t)n * op->ds);
        const void *dsrc = h->mode == STAGE_ZC ? stage_dptr(h, src, (size_t)n * op->ss) : NULL;
        if (ddst != NULL && h->mode == STAGE_ZC && dsrc != NULL) {
            void *q = c->stream[k & 1];
            /* no copies: gpu.h2d and gpu.d2h read 0, gpu.kernel the kernel */
            if (!err && ev) err = pncxrt_event_record(ev[0], q);
            if (!err && ev) err = pncxrt_event_record(ev[1], q);
            if (!err) err = launch_op(op, dsrc, ddst, n, h->want_status ? c->dstatus : NULL, q);
            if (!err && ev) err = pncxrt_event_record(ev[2], q);
            if (!err && ev) err = pncxrt_event_record(ev[3], q);
            if (!err) err = pncxrt_event_record(c->sev_out[e], q);
            PH_ADD(PH_CONV_ENQUEUE, t0);
            if (err) return h->err = err < 0 ? err : PNCX_EDEVICE;
            h->pushed++;
            return k;
        }
        if (ddst != NULL) {
            /* the slot's last reader is chunk k-NDBUF's kernel, on the out stream */
            if (k >= NDBUF) err = pncxrt_stream_wait_event(si, c->sev_out[(k - NDBUF) % NSEV]);
            if (!err && ev) err = pncxrt_event_record(ev[0], si);
            if (!err) err = pncxrt_memcpy_h2d(din, src, (size_t)n * op->ss, si);
            if (!err && ev) err = pncxrt_event_record(ev[1], si);
            if (!err) err = pncxrt_event_record(c->sev_conv[e], si);
            if (!err) err = pncxrt_stream_wait_event(so, c->sev_conv[e]);
            if (!err && ev) err = pncxrt_event_record(ev[2], so);
            if (!err) err = launch_op(op, din, ddst, n, h->want_status ? c->dstatus : NULL, so);
            if (!err && ev) err = pncxrt_event_record(ev[3], so);
            if (!err) err = pncxrt_event_record(c->sev_out[e], so);
            PH_ADD(PH_CONV_ENQUEUE, t0);
            if (err) return h->err = err < 0 ? err : PNCX_EDEVICE;
            h->pushed++;
            return k;
        }
    }
    if (op->ss == op->ds && src == dst) dout = din;            /* in-place swap */
    if (h->mode == STAGE_ALT) {
        /* chunk k wholly on stream k & 1; slot k % NDBUF was last used by
         * chunk k - NDBUF, on the same stream (NDBUF is even) */
        void *q = c->stream[k & 1];
        if (!err && ev) err = pncxrt_event_record(ev[0], q);
        if (!err) err = pncxrt_memcpy_h2d(din, src, (size_t)n * op->ss, q);
        if (!err && h->preserve && dout != din) err = pncxrt_memcpy_h2d(dout, dst, (size_t)n * op->ds, q);
        if (!err && ev) err = pncxrt_event_record(ev[1], q);
        if (!err && !(op->kind == PNCXK_SWAP && op->a == 1 && dout == din))
            err = launch_op(op, din, dout, n, h->want_status ? c->dstatus : NULL, q);
        if (!err && ev) err = pncxrt_event_record(ev[2], q);
        if (!err) err = pncxrt_memcpy_d2h(dst, dout, (size_t)n * op->ds, q);
        if (!err && ev) err = pncxrt_event_record(ev[3], q);
        if (!err) err = pncxrt_event_record(c->sev_out[e], q);
        PH_ADD(PH_CONV_ENQUEUE, t0);
        if (err) return h->err = err < 0 ? err : PNCX_EDEVICE;
        h->pushed++;
        return k;
    }
    /* the slot's previous chunk must be back on the host */
    if (k >= NDBUF) err = pncxrt_stream_wait_event(si, c->sev_out[(k - NDBUF) % NSEV]);
    if (!err && ev) err = pncxrt_event_record(ev[0], si);
    if (!err) err = pncxrt_memcpy_h2d(din, src, (size_t)n * op->ss, si);
    if (!err && h->preserve && dout != din) err = pncxrt_memcpy_h2d(dout, dst, (size_t)n * op->ds, si);
    if (!err && ev) err = pncxrt_event_record(ev[1], si);
    if (!err && !(op->kind == PNCXK_SWAP && op->a == 1 && dout == din))
        err = launch_op(op, din, dout, n, h->want_status ? c->dstatus : NULL, si);
    if (!err) err = pncxrt_event_record(c->sev_conv[e], si);
    if (!err) err = pncxrt_stream_wait_event(so, c->sev_conv[e]);
    if (!err && ev) err = pncxrt_event_record(ev[2], so);
    if (!err) err = pncxrt_memcpy_d2h(dst, dout, (size_t)n * op->ds, so);
    if (!err && ev) err = pncxrt_event_record(ev[3], so);
    if (!err) err = pncxrt_event_record(c->sev_out[e], so);
    PH_ADD(PH_CONV_ENQUEUE, t0);
    if (err) {
        h->err = err < 0 ? err : PNCX_EDEVICE;
        return h->err;
    }
    h->pushed++;
    return k;
}

/* chunk k's result is in its host destination */
int pncx_stage_wait(pncx_stage *h, int k)
{
    int err;
    double t0;
    if (h->err) return h->err;
    if (k < h->waited) return NC_NOERR;
    if (k >= h->pushed || k < h->pushed - NSEV) return NC_EINVAL;
    t0 = PH_T0();
    err = pncxrt_event_sync(h->c->sev_out[k % NSEV]);
    PH_ADD(PH_CONV_SYNC, t0);
    if (err) return h->err = PNCX_EDEVICE;
    h->waited = k + 1;
    return NC_NOERR;
}

/* wait for every chunk, release the context; the call's first status */
int pncx_stage_end(pncx_stage *h)
{
    ctx_t *c;
    int err, st = 0, i;
    double t0;
    if (h == NULL) return NC_NOERR;
    c = h->c;
    err = h->err;
    t0 = PH_T0();
    for (i = 0; i < NSLOT; i++) {                  /* also drains after an error */
        const int e2 = pncxrt_stream_sync(c->stream[i]);
        if (!err && e2) err = PNCX_EDEVICE;
    }
    PH_ADD(PH_CONV_SYNC, t0);
    for (i = 0; i < h->ph_ev && !err; i++) {
        float a = 0, b = 0, d = 0;
        void **ev = &c->pev[4 * i];
        if (pncxrt_event_elapsed_ms(&a, ev[0], ev[1]) || pncxrt_event_elapsed_ms(&b, ev[1], ev[2]) ||
            pncxrt_event_elapsed_ms(&d, ev[2], ev[3]))
            break;
        pncx_ph_add_us(PH_GPU_H2D, 1e3 * a);
        pncx_ph_add_us(PH_GPU_KERNEL, 1e3 * b);
        pncx_ph_add_us(PH_GPU_D2H, 1e3 * d);
    }
    t0 = PH_T0();
    if (!err && h->want_status && h->pushed > 0) {  /* the status word, through pinned memory */
        err = pncxrt_memcpy_d2h(c->hstat, c->dstatus, sizeof(int), c->stream[0]);
        if (!err) err = pncxrt_stream_sync(c->stream[0]);
        if (!err) st = c->hstat[0];
    }
    PH_ADD(PH_CONV_STATUS, t0);
    t0 = PH_T0();
    unpin_all(&h->pn);
    PH_ADD(PH_CONV_UNPIN, t0);
    pthread_mutex_unlock(&c->lock);
    free(h);
    if (err) return err < 0 ? err : PNCX_EDEVICE;
    return st;
}

long long pncx_stage_chunk(const pncx_stage *h) { return h->chunk; }

/* One conversion launch between device-accessible pointers (HBM, pinned or
 * registered host memory, a registered file window), waited for.  Returns
 * the status (NC_ERANGE) or an error. */
int pncx_direct_convert(int dir, int cdf_ver, int xtype, int itype, const void *fillp, const void *dsrc,
                        void *ddst, long long n, void *const *after)
{
    op_t op;
    ctx_t *c;
    int err, st = 0, want;
    double t0 = PH_T0();
    if (dir == PNCX_SWAP_DIR) {
        memset(&op, 0, sizeof op);
        op.kind = PNCXK_SWAP;
        op.a = op.ss = op.ds = xtype;
    } else if ((err = classify(dir, cdf_ver, xtype, itype, fillp, &op)) != NC_NOERR) {
        return err;
    }
    if (n <= 0) return NC_NOERR;
    if (!have_device() || (c = get_ctx()) == NULL) return PNCX_EDEVICE;
    want = op.kind != PNCXK_SWAP;
    pthread_mutex_lock(&c->lock);
    err = stage_slots(c, 0);                      /* the events and the pinned status word */
    if (!err && after != NULL) {
        /* a device buffer the caller's stream produces (put) or still reads
         * (get): the launch follows everything queued there before the call */
        err = pncxrt_event_record(c->sev_init, *after);
        if (!err) err = pncxrt_stream_wait_event(c->stream[0], c->sev_init);
    }
    if (!err && want) err = pncxrt_memset(c->dstatus, 0, sizeof(int), c->stream[0]);
    if (!err) err = launch_op(&op, dsrc, ddst, n, want ? c->dstatus : NULL, c->stream[0]);
    if (!err && want) err = pncxrt_memcpy_d2h(c->hstat, c->dstatus, sizeof(int), c->stream[0]);
    if (!err) err = pncxrt_stream_sync(c->stream[0]);
    if (!err && want) st = c->hstat[0];
    pthread_mutex_unlock(&c->lock);
    PH_ADD(dir == PNCX_GET ? PH_GET_CONVERT : PH_PUT_CONVERT, t0);
    if (err) return err < 0 ? err : PNCX_EDEVICE;
    return st;
}

/* the whole call through a stage: host-buffer entry points */
/* Buffers the caller pinned or registered before a call of 64 MiB or more
 * take SDMA copies on alternating streams: 2 GiB in-place swaps 37-38 GiB/s
 * of slab against 29 zero copy, getn int->double 67 against 61.  Zero copy
 * stays for pageable buffers (pinned by the call: 29.6 against 25-29.5 swap,
 * 61 against 51 getn) and for smaller calls (profiles/r04u_host_modes.txt) */
static int pre_mapped_large(const op_t *op, const void *src, const void *dst, long long n)
{
    const size_t sb = (size_t)n * op->ss, db = (size_t)n * op->ds;
    if (pncx_knob(PNCXK_KNOB_HOST_ZC) >= 0 || sb + db < ((size_t)64 << 20)) return 0;
    return pncxrt_host_dptr_range(src, sb) != NULL && (dst == src || pncxrt_host_dptr_range(dst, db) != NULL);
}

static int host_staged(const op_t *op, const void *src, void *dst, long long n, int preserve)
{
    pncx_stage *h;
    long long off, chunk;
    int err;
    const int alt = pre_mapped_large(op, src, dst, n);
    chunk = stage_chunk_elems(op, n);
    if ((err = stage_open(&h, op, preserve, chunk, n)) != NC_NOERR) return err;
    if (alt) h->mode = STAGE_ALT;
    pin_range(&h->pn, src, (size_t)n * op->ss);
    pin_range(&h->pn, dst, (size_t)n * op->ds);
    if (h->mode == STAGE_ZC || h->mode == STAGE_ZCOUT) {
        pncx_stage_hint(h, src, (size_t)n * op->ss);
        if (dst != src) pncx_stage_hint(h, dst, (size_t)n * op->ds);
    }
    for (off = 0; off < n; off += chunk) {
        const long long m = n - off < chunk ? n - off : chunk;
        const int k = pncx_stage_push(h, (const uint8_t *)src + (size_t)off * op->ss,
                                      (uint8_t *)dst + (size_t)off * op->ds, m);
        if (k < 0) break;
    }
    return pncx_stage_end(h);
}

/* ------------------------------------------------------------------------ */
/* host-buffer entry points                                                  */
/* ------------------------------------------------------------------------ */
int pncx_in_swapn(void *buf, pncx_offset nelems, int esize)
{
    op_t op;
    if (esize <= 1 || nelems <= 0) return NC_NOERR;          /* convert_swap.m4:147 */
    if (!have_device()) return PNCX_EDEVICE;
    memset(&op, 0, sizeof op);
    op.kind = PNCXK_SWAP;
    op.a = esize;
    op.ss = op.ds = esize;
    return host_staged(&op, buf, buf, nelems, 0);
}

int pncx_putn(int cdf_ver, int xtype, void *xbuf, const void *ibuf, pncx_offset nelems,
              int itype, const void *fillp)
{
    op_t op;
    int err = classify(PNCX_PUT, cdf_ver, xtype, itype, fillp, &op);
    if (err != NC_NOERR) return err;
    if (nelems <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    return host_staged(&op, ibuf, xbuf, nelems, op.c);
}

int pncx_getn(int cdf_ver, int xtype, const void *xbuf, void *ibuf, pncx_offset nelems,
              int itype)
{
    op_t op;
    int err = classify(PNCX_GET, cdf_ver, xtype, itype, NULL, &op);
    if (err != NC_NOERR) return err;
    if (nelems <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    return host_staged(&op, xbuf, ibuf, nelems, 0);
}

/* ------------------------------------------------------------------------ */
/* fill path: fill_var_buf (ncmpio_fill.c:89-140)                            */
/* ------------------------------------------------------------------------ */
/* default external fill patterns, big-endian (ncmpio_fill.c:50-60) */
static int default_fill_xvalue(int xtype, unsigned char *out)
{
    static const unsigned char f_char[1] = {0x00}, f_byte[1] = {0x81}, f_short[2] = {0x80, 0x01},
        f_int[4] = {0x80, 0x00, 0x00, 0x01}, f_float[4] = {0x7C, 0xF0, 0x00, 0x00},
        f_double[8] = {0x47, 0x9E, 0, 0, 0, 0, 0, 0}, f_ubyte[1] = {0xFF}, f_ushort[2] = {0xFF, 0xFF},
        f_uint[4] = {0xFF, 0xFF, 0xFF, 0xFF}, f_int64[8] = {0x80, 0, 0, 0, 0, 0, 0, 0x02},
        f_uint64[8] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFE};
    const unsigned char *p;
    switch (xtype) {
        case NC_CHAR: p = f_char; break;
        case NC_BYTE: p = f_byte; break;
        case NC_SHORT: p = f_short; break;
        case NC_INT: p = f_int; break;
        case NC_FLOAT: p = f_float; break;
        case NC_DOUBLE: p = f_double; break;
        case NC_UBYTE: p = f_ubyte; break;
        case NC_USHORT: p = f_ushort; break;
        case NC_UINT: p = f_uint; break;
        case NC_INT64: p = f_int64; break;
        case NC_UINT64: p = f_uint64; break;
        default: return NC_EBADTYPE;
    }
    memcpy(out, p, (size_t)pncx_xlen(xtype));
    return NC_NOERR;
}

int pncx_dev_fill(int xtype, void *dxbuf, pncx_offset nelems, const void *xvalue, pncx_stream_t stream)
{
    unsigned char v[8];
    const int xs = pncx_xlen(xtype);
    if (xs < 0) return NC_EBADTYPE;
    if (xvalue == NULL) {
        if (default_fill_xvalue(xtype, v) != NC_NOERR) return NC_EBADTYPE;
    } else {
        memcpy(v, xvalue, (size_t)xs);
    }
    if (nelems <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    return pncxk_fill(dxbuf, nelems, xs, v, stream);
}

int pncx_fill(int xtype, void *xbuf, pncx_offset nelems, const void *xvalue)
{
    ctx_t *c;
    long long off, chunk;
    int err = 0, slot = 0, i;
    pinned_t pn = {{NULL, NULL}, 0};
    const int xs = pncx_xlen(xtype);
    if (xs < 0) return NC_EBADTYPE;
    if (nelems <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    c = get_ctx();
    if (c == NULL) return PNCX_EDEVICE;
    pthread_mutex_lock(&c->lock);
    pin_range(&pn, xbuf, (size_t)nelems * xs);
    chunk = (long long)(chunk_bytes() / (size_t)xs);
    if (chunk > nelems) chunk = nelems;
    err = ensure_dbuf(c, ALIGN16((size_t)chunk * xs));
    /* the pattern is generated once per slot and streamed out chunk by chunk */
    for (i = 0; i < NSLOT && !err; i++)
        err = pncx_dev_fill(xtype, c->dbuf[i], chunk, xvalue, c->stream[i]);
    for (off = 0; off < nelems && !err; off += chunk, slot ^= 1) {
        const long long m = nelems - off < chunk ? nelems - off : chunk;
        err = pncxrt_memcpy_d2h((uint8_t *)xbuf + (size_t)off * xs, c->dbuf[slot], (size_t)m * xs, c->stream[slot]);
    }
    for (i = 0; i < NSLOT; i++) {
        int e2 = pncxrt_stream_sync(c->stream[i]);
        if (!err && e2) err = e2;
    }
    unpin_all(&pn);
    pthread_mutex_unlock(&c->lock);
    return err ? (err < 0 ? err : PNCX_EDEVICE) : NC_NOERR;
}

/* ------------------------------------------------------------------------ */
/* varm (imap) fused gather/scatter + conversion                             */
/* ------------------------------------------------------------------------ */
/* Mirrors ncmpii_create_imaptype (create_imaptype.c:25-139): returns 1 with
 * *n = number of elements when imap[] is a true (non-contiguous) varm layout,
 * 0 when it is plain C order (then the contiguous kernels apply). */
static int imap_layout(int ndims, const pncx_offset *count, const pncx_offset *imap, pncxk_imap *m,
                       long long *n, long long *span, int *err)
{
    int d;
    long long blk = 1, total = 1, sp = 0;
    *err = NC_NOERR;
    if (ndims < 0 || ndims > PNCX_MAX_DIMS) { *err = NC_EINVAL; return 0; }
    memset(m, 0, sizeof *m);
    for (d = 0; d < ndims; d++) {
        if (count[d] < 0 || (imap != NULL && imap[d] < 0)) { *err = NC_EINVAL; return 0; }
        total *= count[d];
    }
    *n = total;
    if (imap == NULL || ndims == 0 || total <= 1) { *span = total; return 0; }
    d = ndims;
    while (--d >= 0 && blk == imap[d]) blk *= count[d];
    if (d == -1) { *span = total; return 0; }       /* contiguous layout */
    m->ndims = ndims;
    for (d = 0; d < ndims; d++) {
        m->count[d] = count[d];
        m->imap[d] = imap[d];
        if (count[d] > m->max_count) m->max_count = count[d];
        sp += (count[d] - 1) * imap[d];
    }
    *span = total ? sp + 1 : 0;
    return 1;
}

static int launch_imap_op(const op_t *op, const void *src, void *dst, long long n, const pncxk_imap *m,
                          int gather, int *dstatus, void *stream)
{
    pncxk_args a;
    a.src = src;
    a.dst = dst;
    a.n = n;
    a.fill = op->fill;
    a.status = dstatus;
    a.stream = stream;
    a.nontemporal = nontemporal_mode();
    return pncxk_launch_imap(op->kind, op->a, op->b, op->c, &a, m, gather);
}

int pncx_dev_putn_imap(int cdf_ver, int xtype, void *dxbuf, const void *dibuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, int itype,
                       const void *fillp, int *dstatus, pncx_stream_t stream)
{
    op_t op;
    pncxk_imap m;
    long long n, span;
    int err = classify(PNCX_PUT, cdf_ver, xtype, itype, fillp, &op), e2;
    if (err != NC_NOERR) return err;
    if (!imap_layout(ndims, count, imap, &m, &n, &span, &e2)) {
        if (e2 != NC_NOERR) return e2;
        return pncx_dev_putn(cdf_ver, xtype, dxbuf, dibuf, n, itype, fillp, dstatus, stream);
    }
    if (n <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    return launch_imap_op(&op, dibuf, dxbuf, n, &m, 1, dstatus, stream);
}

int pncx_dev_getn_imap(int cdf_ver, int xtype, const void *dxbuf, void *dibuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, int itype,
                       int *dstatus, pncx_stream_t stream)
{
    op_t op;
    pncxk_imap m;
    long long n, span;
    int err = classify(PNCX_GET, cdf_ver, xtype, itype, NULL, &op), e2;
    if (err != NC_NOERR) return err;
    if (!imap_layout(ndims, count, imap, &m, &n, &span, &e2)) {
        if (e2 != NC_NOERR) return e2;
        return pncx_dev_getn(cdf_ver, xtype, dxbuf, dibuf, n, itype, dstatus, stream);
    }
    if (n <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    return launch_imap_op(&op, dxbuf, dibuf, n, &m, 0, dstatus, stream);
}

/* host varm: stage the user-buffer span and the packed buffer in one slot */
static int host_imap(int dir, int cdf_ver, int xtype, void *xbuf, void *ibuf, int ndims,
                     const pncx_offset *count, const pncx_offset *imap, int itype, const void *fillp)
{
    op_t op;
    pncxk_imap m;
    long long n, span;
    ctx_t *c;
    int err = classify(dir, cdf_ver, xtype, itype, fillp, &op), e2, st = 0;
    pinned_t pn = {{NULL, NULL}, 0};
    size_t xs, is, xb, ib;
    uint8_t *dx, *di;
    void *s;
    if (err != NC_NOERR) return err;
    if (!imap_layout(ndims, count, imap, &m, &n, &span, &e2)) {
        if (e2 != NC_NOERR) return e2;
        return dir == PNCX_PUT ? pncx_putn(cdf_ver, xtype, xbuf, ibuf, n, itype, fillp)
                               : pncx_getn(cdf_ver, xtype, xbuf, ibuf, n, itype);
    }
    if (n <= 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    c = get_ctx();
    if (c == NULL) return PNCX_EDEVICE;
    xs = (size_t)pncx_xlen(xtype);
    is = (size_t)pncx_ilen(itype);
    xb = ALIGN16((size_t)n * xs);
    ib = ALIGN16((size_t)span * is);
    pthread_mutex_lock(&c->lock);
    pin_range(&pn, ibuf, (size_t)span * is);
    pin_range(&pn, xbuf, (size_t)n * xs);
    s = c->stream[0];
    err = ensure_dbuf(c, xb + ib);
    dx = (uint8_t *)c->dbuf[0];
    di = dx + xb;
    if (!err) err = pncxrt_memset(c->dstatus, 0, sizeof(int), s);
    if (!err) err = pncxrt_memcpy_h2d(di, ibuf, (size_t)span * is, s);     /* user span */
    if (dir == PNCX_PUT) {
        if (!err && op.c) err = pncxrt_memcpy_h2d(dx, xbuf, (size_t)n * xs, s);
        if (!err) err = launch_imap_op(&op, di, dx, n, &m, 1, c->dstatus, s);
        if (!err) err = pncxrt_memcpy_d2h(xbuf, dx, (size_t)n * xs, s);
    } else {
        if (!err) err = pncxrt_memcpy_h2d(dx, xbuf, (size_t)n * xs, s);
        if (!err) err = launch_imap_op(&op, dx, di, n, &m, 0, c->dstatus, s);
        if (!err) err = pncxrt_memcpy_d2h(ibuf, di, (size_t)span * is, s);
    }
    if (!err) err = pncxrt_memcpy_d2h(&st, c->dstatus, sizeof(int), s);
    if (!err) err = pncxrt_stream_sync(s);
    unpin_all(&pn);
    pthread_mutex_unlock(&c->lock);
    if (err) return err < 0 ? err : PNCX_EDEVICE;
    return st;
}

int pncx_putn_imap(int cdf_ver, int xtype, void *xbuf, const void *ibuf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, int itype, const void *fillp)
{
    return host_imap(PNCX_PUT, cdf_ver, xtype, xbuf, (void *)ibuf, ndims, count, imap, itype, fillp);
}

int pncx_getn_imap(int cdf_ver, int xtype, const void *xbuf, void *ibuf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, int itype)
{
    return host_imap(PNCX_GET, cdf_ver, xtype, (void *)xbuf, ibuf, ndims, count, imap, itype, NULL);
}

/* ------------------------------------------------------------------------ */
/* ncmpidiff data comparison                                                  */
/* ------------------------------------------------------------------------ */
int pncx_dev_first_diff(const void *da, const void *db, pncx_offset nelems, int itype, int tolerance,
                        double tol_diff, double tol_ratio, pncx_offset *first, pncx_stream_t stream)
{
    ctx_t *c;
    unsigned long long h = ~0ULL;
    int err;
    if (first == NULL || pncx_ilen(itype) < 0) return first == NULL ? NC_EINVAL : NC_EBADTYPE;
    *first = -1;
    if (nelems <= 0) return NC_NOERR;
    if (!have_device() || (c = get_ctx()) == NULL) return PNCX_EDEVICE;
    pthread_mutex_lock(&c->lock);
    if (c->dfirst == NULL && pncxrt_malloc((void **)&c->dfirst, sizeof(unsigned long long)) != 0) {
        pthread_mutex_unlock(&c->lock);
        return PNCX_EDEVICE;
    }
    err = pncxrt_memset(c->dfirst, 0xff, sizeof(unsigned long long), stream);
    if (!err) err = pncxk_first_diff(da, db, nelems, itype, tolerance, tol_diff, tol_ratio, c->dfirst, stream);
    if (!err) err = pncxrt_memcpy_d2h(&h, c->dfirst, sizeof h, stream);
    if (!err) err = pncxrt_stream_sync(stream);
    pthread_mutex_unlock(&c->lock);
    if (err) return err < 0 ? err : PNCX_EDEVICE;
    *first = h == ~0ULL ? -1 : (pncx_offset)h;
    return NC_NOERR;
}

/* ------------------------------------------------------------------------ */
/* derived buftypes: committed flattened typemaps, pack/unpack fused into    */
/* the imap gather/scatter kernel (pncx_kern.hpp tmap_byte)                  */
/* ------------------------------------------------------------------------ */
struct pncx_dtype {
    int        itype, isz, layout;
    int        refs;
    long long  tn, extent, nblk;
    long long  lo, hi;                /* byte bounds of one copy: [lo, hi)     */
    long long  len, stride, disp0;    /* layout 0/1                            */
    long long *pre, *disp;            /* host table (nblk each)                */
    long long *dtab;                  /* device: pieces of the runs (<= PNCX_TMAP_PIECE
                                       * elements): pre[np + 1], disp[np], then
                                       * cidx[nq + 1], the piece of element 64q */
    long long  np, nq;                /* pieces, 64-element chunks             */
    int        runmajor;              /* runs long enough for one wave each    */
    unsigned  *doff;                  /* device: byte offset - lo of each element
                                       * of a copy (short-run tables, tmode 4), or
                                       * (off16) one base per 64-element chunk
                                       * followed by 16-bit offsets from it (tmode 5) */
    int        off16;                 /* map width: 0 = 32-bit, 1 = 16-bit, 2 = 8-bit gap counts,
                                       * 3 = 4-bit gap steps */
    long long  rn1, rn2, rs1, rs2;    /* table runs on a 2-level lattice: run i at
                                       * disp0 + (i % rn1)*rs1 + (i / rn1)*rs2 bytes
                                       * (rn1 = 0: not one) */
    struct pncx_dtype *bytes;         /* the same typemap in bytes (pncx_dev_pack), made on first use */
    pthread_mutex_t bytes_lock;
};

/* Largest typemap (elements per copy) that gets a per-element offset map:
 * 4 B of HBM per element, read coalesced, instead of a table search per
 * element.  PNCX_TOFF_MAX_ELEMS overrides (0 disables; read at commit). */
static long long toff_max_elems(void)
{
    const long long v = pncx_knob(PNCXK_KNOB_TOFF_MAX_ELEMS);
    return v >= 0 ? v : (1LL << 26);
}

int pncx_type_commit(int itype, pncx_offset nblocks, const pncx_offset *disp,
                     const pncx_offset *blocklen, pncx_offset extent, pncx_dtype **dtype)
{
    pncx_dtype *t;
    long long i, k = 0, *len;
    const int isz = pncx_ilen(itype);
    if (dtype == NULL) return NC_EINVAL;
    *dtype = NULL;
    if (isz < 0) return NC_EBADTYPE;
    if (nblocks < 0 || (nblocks > 0 && (disp == NULL || blocklen == NULL))) return NC_EINVAL;
    for (i = 0; i < nblocks; i++)
        if (blocklen[i] < 0) return NC_EINVAL;
    t = (pncx_dtype *)calloc(1, sizeof *t);
    len = (long long *)malloc(sizeof(long long) * (size_t)(nblocks ? nblocks : 1));
    if (t != NULL) {
        t->pre = (long long *)malloc(sizeof(long long) * (size_t)(nblocks ? nblocks : 1));
        t->disp = (long long *)malloc(sizeof(long long) * (size_t)(nblocks ? nblocks : 1));
    }
    if (t == NULL || len == NULL || t->pre == NULL || t->disp == NULL) {
        if (t) { free(t->pre); free(t->disp); }
        free(t);
        free(len);
        return NC_ENOMEM;
    }
    t->itype = itype;
    t->isz = isz;
    t->extent = extent;
    t->refs = 1;
    pthread_mutex_init(&t->bytes_lock, NULL);
    /* normalise: drop empty runs, merge runs that continue each other */
    for (i = 0; i < nblocks; i++) {
        if (blocklen[i] == 0) continue;
        if (k > 0 && t->disp[k - 1] + len[k - 1] * isz == disp[i]) { len[k - 1] += blocklen[i]; continue; }
        t->disp[k] = disp[i];
        len[k++] = blocklen[i];
    }
    t->nblk = k;
    for (i = 0; i < k; i++) {
        const long long end = t->disp[i] + len[i] * isz;
        t->pre[i] = t->tn;
        t->tn += len[i];
        if (i == 0 || t->disp[i] < t->lo) t->lo = t->disp[i];
        if (i == 0 || end > t->hi) t->hi = end;
    }
    if (k == 0 || (k == 1 && extent == len[0] * isz)) {
        t->layout = 0;                                   /* contiguous */
        t->disp0 = k ? t->disp[0] : 0;
        t->len = k ? len[0] : 0;
    } else {
        int uniform = 1;
        for (i = 1; i < k && uniform; i++)
            uniform = len[i] == len[0] && t->disp[i] - t->disp[i - 1] == t->disp[1] - t->disp[0];
        t->len = len[0];
        t->disp0 = t->disp[0];
        t->stride = k > 1 ? t->disp[1] - t->disp[0] : 0;
        t->layout = uniform ? 1 : 2;
    }
    /* a table whose equal-length runs sit on a 2-level lattice (a 3-D
     * subarray: rows, then planes) is also an imap; flex_layout can then take
     * the varm kernels (k_imap_rows) instead of the run-piece kernel */
    if (t->layout == 2 && k > 2) {
        long long n1 = 1, i2;
        int ok = 1;
        const long long s1 = t->disp[1] - t->disp[0];
        for (i = 1; i < k && ok; i++) ok = len[i] == len[0];
        while (n1 < k && t->disp[n1] - t->disp[n1 - 1] == s1) n1++;
        ok = ok && n1 > 1 && n1 < k && k % n1 == 0 && s1 > 0;
        if (ok) {
            const long long s2 = t->disp[n1] - t->disp[0];
            for (i2 = 0; i2 < k && ok; i2++)
                ok = t->disp[i2] == t->disp[0] + (i2 % n1) * s1 + (i2 / n1) * s2;
            ok = ok && s2 > 0 && s1 % isz == 0 && s2 % isz == 0 && t->disp[0] % isz == 0 && extent % isz == 0;
            if (ok) {
                t->rn1 = n1;
                t->rn2 = k / n1;
                t->rs1 = s1;
                t->rs2 = s2;
            }
        }
    }
    free(len);
    if (t->layout == 2 && have_device()) {
        /* The general table lives in HBM from now on (device calls stay
         * async), with runs split into pieces of at most PNCX_TMAP_PIECE
         * elements: in packed order a wave then takes one piece when runs
         * average >= 48 elements (k_tmap_runs), else lanes search the table. */
        long long np = 0, p, e, nq, q;
        int derr = 0;
        long long *h;
        for (i = 0; i < k; i++) {
            const long long ln = (i + 1 < k ? t->pre[i + 1] : t->tn) - t->pre[i];
            np += (ln + PNCX_TMAP_PIECE - 1) / PNCX_TMAP_PIECE;
        }
        nq = (t->tn + 63) / 64;
        h = (long long *)malloc(sizeof(long long) * (size_t)(2 * np + 1 + nq + 1));
        if (h == NULL) derr = NC_ENOMEM;
        for (i = 0, p = 0; i < k && !derr; i++) {
            const long long ln = (i + 1 < k ? t->pre[i + 1] : t->tn) - t->pre[i];
            for (e = 0; e < ln; e += PNCX_TMAP_PIECE, p++) {
                h[p] = t->pre[i] + e;
                h[np + 1 + p] = t->disp[i] + e * isz;
            }
        }
        if (!derr) {
            long long *cidx = h + 2 * np + 1;
            h[np] = t->tn;
            for (q = 0, p = 0; q < nq; q++) {         /* piece holding element 64q */
                while (p + 1 < np && h[p + 1] <= 64 * q) p++;
                cidx[q] = p;
            }
            cidx[nq] = np - 1;
            t->np = np;
            t->nq = nq;
            t->runmajor = t->tn >= 48 * k;
            if (pncxrt_malloc((void **)&t->dtab, sizeof(long long) * (size_t)(2 * np + 1 + nq + 1)) != 0 ||
                pncxrt_memcpy_h2d(t->dtab, h, sizeof(long long) * (size_t)(2 * np + 1 + nq + 1), NULL) != 0 ||
                pncxrt_stream_sync(NULL) != 0)
                derr = PNCX_EDEVICE;
        }
        free(h);
        if (!derr && !t->runmajor && t->tn <= toff_max_elems() && t->hi - t->lo <= 0xffffffffLL) {
            /* short runs: per-element map (offsets from lo fit 32 bits).
             * When every 64-element chunk spans under 64 KiB the map is a
             * 32-bit base per chunk plus 16-bit offsets: 2 B of HBM per
             * element instead of 4 (PNCX_TOFF16=0 keeps 32 bits) */
            unsigned *o = (unsigned *)malloc(sizeof(unsigned) * (size_t)t->tn);
            const long long k16 = pncx_knob(PNCXK_KNOB_TOFF16);
            size_t bytes = sizeof(unsigned) * (size_t)t->tn;
            void *up = o;
            if (o == NULL) derr = NC_ENOMEM;
            for (i = 0; i < k && !derr; i++) {
                const long long ln = (i + 1 < k ? t->pre[i + 1] : t->tn) - t->pre[i];
                for (e = 0; e < ln; e++) o[t->pre[i] + e] = (unsigned)(t->disp[i] - t->lo + e * isz);
            }
            if (!derr && (k16 < 0 || k16 == 4)) {
                /* 4-bit map (tmode 7): a nibble per element, the gap
                 * elements between it and the element before it in its
                 * chunk (0 at a chunk's first), 32 B per chunk after the
                 * chunk bases (padded to 8 bases: the nibbles stay 32-byte
                 * aligned) -- 0.5 B per element for typemaps whose runs
                 * rise through each chunk with gaps of at most 15 elements.
                 * k_tgap sums a chunk's nibbles across the wave */
                const long long nq4 = (t->tn + 63) / 64, nqp = (nq4 + 7) & ~7LL;
                unsigned *base = (unsigned *)calloc(1, sizeof(unsigned) * (size_t)nqp + 32 * (size_t)nq4);
                int fits = base != NULL;
                unsigned char *d4 = fits ? (unsigned char *)(base + nqp) : NULL;
                for (e = 0; e < t->tn && fits; e++) {
                    if ((e & 63) == 0) {
                        base[e >> 6] = o[e];
                        continue;
                    }
                    fits = o[e] > o[e - 1] && (o[e] - o[e - 1]) % (unsigned)isz == 0 &&
                           (o[e] - o[e - 1]) / (unsigned)isz <= 16;
                    if (fits) d4[e >> 1] |= (unsigned char)(((o[e] - o[e - 1]) / (unsigned)isz - 1) << ((e & 1) * 4));
                }
                if (fits) {
                    bytes = sizeof(unsigned) * (size_t)nqp + 32 * (size_t)nq4;
                    up = base;
                    t->off16 = 3;
                } else {
                    free(base);
                }
            }
            if (!derr && k16 != 0 && k16 != 16 && t->off16 == 0) {
                /* 8-bit map (tmode 6): element e of chunk q sits ((e & 63) +
                 * g[e]) elements past the chunk's first element, g counting
                 * the gap elements before it in the chunk -- 1 B per element
                 * for typemaps whose offsets rise through each chunk by
                 * whole elements with under 256 gap elements */
                const long long nq8 = (t->tn + 63) / 64;
                unsigned *base = (unsigned *)malloc(sizeof(unsigned) * (size_t)nq8 + (size_t)t->tn);
                int fits = base != NULL;
                unsigned char *d8 = fits ? (unsigned char *)(base + nq8) : NULL;
                for (e = 0; e < t->tn && fits; e++) {
                    const unsigned b0 = o[e & ~63LL];
                    long long g;
                    if ((e & 63) == 0) base[e >> 6] = b0;
                    fits = o[e] >= b0 && (o[e] - b0) % (unsigned)isz == 0;
                    g = (long long)((o[e] - b0) / (unsigned)isz) - (e & 63);
                    fits = fits && g >= 0 && g <= 255;
                    if (fits) d8[e] = (unsigned char)g;
                }
                if (fits) {
                    bytes = sizeof(unsigned) * (size_t)nq8 + (size_t)t->tn;
                    up = base;
                    t->off16 = 2;
                } else {
                    free(base);
                }
            }
            if (!derr && k16 != 0 && t->off16 == 0) {
                const long long nq16 = (t->tn + 63) / 64;
                unsigned *base = (unsigned *)malloc(sizeof(unsigned) * (size_t)nq16 + sizeof(unsigned short) * (size_t)t->tn);
                int fits = base != NULL;
                for (q = 0; q < nq16 && fits; q++) {
                    const long long r1 = 64 * q + 64 < t->tn ? 64 * q + 64 : t->tn;
                    unsigned mn = o[64 * q], mx = o[64 * q];
                    for (e = 64 * q + 1; e < r1; e++) {
                        if (o[e] < mn) mn = o[e];
                        if (o[e] > mx) mx = o[e];
                    }
                    base[q] = mn;
                    fits = mx - mn <= 0xffffu;
                }
                if (fits) {
                    unsigned short *d16 = (unsigned short *)(base + nq16);
                    for (e = 0; e < t->tn; e++) d16[e] = (unsigned short)(o[e] - base[e >> 6]);
                    bytes = sizeof(unsigned) * (size_t)nq16 + sizeof(unsigned short) * (size_t)t->tn;
                    up = base;
                    t->off16 = 1;
                } else {
                    free(base);
                }
            }
            if (!derr && (pncxrt_malloc((void **)&t->doff, bytes) != 0 ||
                          pncxrt_memcpy_h2d(t->doff, up, bytes, NULL) != 0 ||
                          pncxrt_stream_sync(NULL) != 0))
                derr = PNCX_EDEVICE;
            if (up != o) free(up);
            free(o);
        }
        if (derr) {
            pncxrt_free(t->doff);
            pncxrt_free(t->dtab);
            free(t->pre);
            free(t->disp);
            free(t);
            return derr;
        }
    }
    *dtype = t;
    return NC_NOERR;
}

/* reference counting: requests that hold a dtype until wait use these */
pncx_dtype *pncx_type_ref(pncx_dtype *t)
{
    if (t) __atomic_add_fetch(&t->refs, 1, __ATOMIC_ACQ_REL);
    return t;
}

int pncx_type_free(pncx_dtype *t)
{
    if (t == NULL) return NC_EINVAL;
    if (__atomic_sub_fetch(&t->refs, 1, __ATOMIC_ACQ_REL) > 0) return NC_NOERR;
    if (t->dtab || t->doff) {
        pncxrt_stream_sync(NULL);
        pncxrt_free(t->dtab);
        pncxrt_free(t->doff);
    }
    if (t->bytes) pncx_type_free(t->bytes);
    pthread_mutex_destroy(&t->bytes_lock);
    free(t->pre);
    free(t->disp);
    free(t);
    return NC_NOERR;
}

/* 1 when bufcount copies of t are one contiguous run, starting *lo bytes in */
int pncx_type_contig(const pncx_dtype *t, long long bufcount, long long *lo)
{
    *lo = t->nblk ? t->disp0 : 0;
    return t->layout == 0 || (t->nblk == 1 && bufcount == 1);
}

int pncx_type_inq(const pncx_dtype *t, int *itype, pncx_offset *nelems, pncx_offset *extent, int *layout)
{
    if (t == NULL) return NC_EINVAL;
    if (itype) *itype = t->itype;
    if (nelems) *nelems = t->tn;
    if (extent) *extent = t->extent;
    if (layout) *layout = t->layout;
    return NC_NOERR;
}

/*
 * Layout of one flexible call.  Returns 0 when the bufcount copies are one
 * contiguous run starting *base bytes after buf (then the plain / imap kernels
 * apply), 1 when the fused typemap kernel is needed (m filled, user bytes in
 * [*lo, *hi) relative to buf), -1 with *err set on a bad argument.
 */
/* elements of one 16-byte vector of the conversion (0: the NULL-fill
 * codecs, which k_imap_rows does not take) */
static int flex_vec(const op_t *op)
{
    const int w = op->ss > op->ds ? op->ss : op->ds;
    return op->c || w <= 0 ? 0 : 16 / w;
}

/* PNCX_TMAP_IMAP=0 keeps lattice tables on the run-piece kernel (A/B) */
static int tmap_imap_enabled(void) { return pncx_knob(PNCXK_KNOB_TMAP_IMAP) != 0; }

/* vec: elements per 16-byte vector of the call's conversion (0: none);
 * *koff: bytes to add to the user pointer handed to the kernel */
static int flex_layout(int ndims, const pncx_offset *count, const pncx_offset *imap, long long bufcount,
                       const pncx_dtype *t, pncxk_imap *m, long long *n, long long *lo, long long *hi,
                       int *err, int vec, long long *koff)
{
    *koff = 0;
    long long span;
    *lo = *hi = 0;
    if (t == NULL || bufcount < 0) { *err = NC_EINVAL; return -1; }
    int packed_order = 0;
    if (!imap_layout(ndims, count, imap, m, n, &span, err)) {
        if (*err != NC_NOERR) return -1;
        m->ndims = 1;                     /* packed order: offset = k */
        m->count[0] = *n;
        m->imap[0] = 1;
        m->max_count = *n;
        packed_order = 1;
    }
    if (bufcount * t->tn != *n) { *err = NC_EIOMISMATCH; return -1; }   /* dtype_decode.c:690 */
    if (t->layout == 0 || (t->nblk == 1 && bufcount == 1)) {
        *lo = t->nblk ? t->disp0 : 0;
        return 0;
    }
    if (packed_order && t->layout == 2 && t->rn1 > 0 && vec > 1 && t->len % vec == 0 && tmap_imap_enabled()) {
        /* lattice table over a contiguous count: copies x planes x rows x
         * run, as an imap from the first run (k_imap_rows) */
        const long long isz = t->isz;
        m->ndims = 4;
        m->count[0] = bufcount; m->count[1] = t->rn2; m->count[2] = t->rn1; m->count[3] = t->len;
        m->imap[0] = t->extent / isz; m->imap[1] = t->rs2 / isz; m->imap[2] = t->rs1 / isz; m->imap[3] = 1;
        m->max_count = bufcount > t->rn2 ? bufcount : t->rn2;
        if (t->rn1 > m->max_count) m->max_count = t->rn1;
        if (t->len > m->max_count) m->max_count = t->len;
        m->tmode = 0;
        *koff = t->disp0;
        {
            const long long last = (bufcount - 1) * t->extent;
            *lo = t->lo < last + t->lo ? t->lo : last + t->lo;
            *hi = t->hi > last + t->hi ? t->hi : last + t->hi;
        }
        return 1;
    }
    m->tmode = t->layout == 2 && t->runmajor && packed_order ? 3
             : t->layout == 2 && t->doff ? (t->off16 == 3 ? 7 : t->off16 == 2 ? 6 : t->off16 ? 5 : 4) : t->layout;
    m->toff = t->doff;
    m->toff16 = t->off16 == 1 ? (const unsigned short *)(t->doff + (t->tn + 63) / 64) : NULL;
    m->toff8 = t->off16 == 2   ? (const unsigned char *)(t->doff + (t->tn + 63) / 64)
             : t->off16 == 3 ? (const unsigned char *)(t->doff + (((t->tn + 63) / 64 + 7) & ~7LL))
                             : NULL;
    m->tlo = t->lo;
    m->tn = t->tn;
    m->textent = t->extent;
    m->tlen = t->len;
    m->tstride = t->stride;
    m->tdisp0 = t->disp0;
    m->tnblk = t->layout == 2 ? t->np : t->nblk;
    m->tpre = t->dtab;
    m->tdisp = t->dtab ? t->dtab + t->np + 1 : NULL;
    m->tcidx = t->dtab ? t->dtab + 2 * t->np + 1 : NULL;
    {
        const long long last = (bufcount - 1) * t->extent;
        *lo = t->lo < last + t->lo ? t->lo : last + t->lo;
        *hi = t->hi > last + t->hi ? t->hi : last + t->hi;
    }
    return 1;
}

int pncx_dev_putn_flex(int cdf_ver, int xtype, void *dxbuf, const void *dbuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                       const pncx_dtype *bt, const void *fillp, int *dstatus, pncx_stream_t stream)
{
    op_t op;
    pncxk_imap m;
    long long n, lo, hi, koff;
    int err, r;
    if (bt == NULL) return NC_EINVAL;
    if ((err = classify(PNCX_PUT, cdf_ver, xtype, bt->itype, fillp, &op)) != NC_NOERR) return err;
    if ((r = flex_layout(ndims, count, imap, bufcount, bt, &m, &n, &lo, &hi, &err, flex_vec(&op), &koff)) < 0)
        return err;
    if (r == 0)
        return pncx_dev_putn_imap(cdf_ver, xtype, dxbuf, (const char *)dbuf + lo, ndims, count, imap,
                                  bt->itype, fillp, dstatus, stream);
    if (n <= 0) return NC_NOERR;
    if (!have_device() || (m.tmode >= 2 && m.tpre == NULL)) return PNCX_EDEVICE;
    return launch_imap_op(&op, (const char *)dbuf + koff, dxbuf, n, &m, 1, dstatus, stream);
}

/* the typemap of t with its runs counted in bytes: MPI_Pack of itype
 * elements is a byte copy over these runs (no conversion) */
static const pncx_dtype *type_bytes(pncx_dtype *t)
{
    pthread_mutex_lock(&t->bytes_lock);
    if (t->bytes == NULL && t->itype != PNCX_ITYPE_UCHAR) {
        long long *bl = (long long *)malloc(sizeof(long long) * (size_t)(t->nblk ? t->nblk : 1)), i;
        if (bl != NULL) {
            for (i = 0; i < t->nblk; i++) bl[i] = ((i + 1 < t->nblk ? t->pre[i + 1] : t->tn) - t->pre[i]) * t->isz;
            if (pncx_type_commit(PNCX_ITYPE_UCHAR, t->nblk, t->disp, bl, t->extent, &t->bytes) != NC_NOERR)
                t->bytes = NULL;
            free(bl);
        }
    }
    pthread_mutex_unlock(&t->bytes_lock);
    return t->itype == PNCX_ITYPE_UCHAR ? t : t->bytes;
}

/* MPI_Pack / MPI_Unpack in HBM (ncmpio_pack_xbuf's first step,
 * ncmpio_util.c:620-652; ncmpio_unpack_xbuf's last, :889-933): a byte copy
 * of the typemap's runs through the typemap kernels (uchar -> NC_UBYTE is a
 * copy in convert_swap.m4's classification). */
static int dev_pack_dir(int pack, void *dpacked, void *dbuf, pncx_offset bufcount, const pncx_dtype *bt,
                        pncx_stream_t stream)
{
    const pncx_dtype *tb;
    pncx_offset cnt;
    int err;
    if (bt == NULL || bufcount < 0) return NC_EINVAL;
    if (bufcount == 0 || bt->tn == 0) return NC_NOERR;
    if (!have_device()) return PNCX_EDEVICE;
    if ((tb = type_bytes((pncx_dtype *)bt)) == NULL) return NC_ENOMEM;
    cnt = bufcount * bt->tn * bt->isz;
    err = pack ? pncx_dev_putn_flex(PNCX_FORMAT_CDF5, NC_UBYTE, dpacked, dbuf, 1, &cnt, NULL, bufcount, tb, NULL,
                                    NULL, stream)
               : pncx_dev_getn_flex(PNCX_FORMAT_CDF5, NC_UBYTE, dpacked, dbuf, 1, &cnt, NULL, bufcount, tb, NULL,
                                    stream);
    if (!err && stream == NULL) err = pncxrt_stream_sync(NULL);
    return err;
}

int pncx_dev_pack(void *dpacked, const void *dbuf, pncx_offset bufcount, const pncx_dtype *buftype,
                  pncx_stream_t stream)
{
    return dev_pack_dir(1, dpacked, (void *)dbuf, bufcount, buftype, stream);
}

int pncx_dev_unpack(const void *dpacked, void *dbuf, pncx_offset bufcount, const pncx_dtype *buftype,
                    pncx_stream_t stream)
{
    return dev_pack_dir(0, (void *)dpacked, dbuf, bufcount, buftype, stream);
}

void *pncx_dev_alloc(pncx_offset nbytes)
{
    void *p = NULL;
    if (nbytes < 0 || !have_device()) return NULL;
    return pncxrt_malloc(&p, (size_t)nbytes) == 0 ? p : NULL;
}

int pncx_dev_free(void *p)
{
    if (p == NULL) return NC_NOERR;
    return pncxrt_free(p) == 0 ? NC_NOERR : PNCX_EDEVICE;
}

int pncx_dev_getn_flex(int cdf_ver, int xtype, const void *dxbuf, void *dbuf, int ndims,
                       const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                       const pncx_dtype *bt, int *dstatus, pncx_stream_t stream)
{
    op_t op;
    pncxk_imap m;
    long long n, lo, hi, koff;
    int err, r;
    if (bt == NULL) return NC_EINVAL;
    if ((err = classify(PNCX_GET, cdf_ver, xtype, bt->itype, NULL, &op)) != NC_NOERR) return err;
    if ((r = flex_layout(ndims, count, imap, bufcount, bt, &m, &n, &lo, &hi, &err, flex_vec(&op), &koff)) < 0)
        return err;
    if (r == 0)
        return pncx_dev_getn_imap(cdf_ver, xtype, dxbuf, (char *)dbuf + lo, ndims, count, imap,
                                  bt->itype, dstatus, stream);
    if (n <= 0) return NC_NOERR;
    if (!have_device() || (m.tmode >= 2 && m.tpre == NULL)) return PNCX_EDEVICE;
    return launch_imap_op(&op, dxbuf, (char *)dbuf + koff, n, &m, 0, dstatus, stream);
}

/* host buffers: stage the user byte span [lo, hi) and the packed buffer */
static int host_flex(int dir, int cdf_ver, int xtype, void *xbuf, void *buf, int ndims,
                     const pncx_offset *count, const pncx_offset *imap, long long bufcount,
                     const pncx_dtype *bt, const void *fillp)
{
    op_t op;
    pncxk_imap m;
    long long n, lo, hi, koff;
    ctx_t *c;
    int err, r, st = 0;
    pinned_t pn = {{NULL, NULL}, 0};
    size_t xs, xb, ub;
    uint8_t *dx, *du, *ubase;
    void *s;
    if (bt == NULL) return NC_EINVAL;
    if ((err = classify(dir, cdf_ver, xtype, bt->itype, fillp, &op)) != NC_NOERR) return err;
    if ((r = flex_layout(ndims, count, imap, bufcount, bt, &m, &n, &lo, &hi, &err, flex_vec(&op), &koff)) < 0)
        return err;
    if (r == 0)
        return dir == PNCX_PUT
                   ? pncx_putn_imap(cdf_ver, xtype, xbuf, (const char *)buf + lo, ndims, count, imap, bt->itype, fillp)
                   : pncx_getn_imap(cdf_ver, xtype, xbuf, (char *)buf + lo, ndims, count, imap, bt->itype);
    if (n <= 0) return NC_NOERR;
    if (!have_device() || (m.tmode >= 2 && m.tpre == NULL)) return PNCX_EDEVICE;
    c = get_ctx();
    if (c == NULL) return PNCX_EDEVICE;
    xs = (size_t)pncx_xlen(xtype);
    xb = ALIGN16((size_t)n * xs);
    ub = (size_t)(hi - lo);
    ubase = (uint8_t *)buf + lo;
    pthread_mutex_lock(&c->lock);
    pin_range(&pn, ubase, ub);
    pin_range(&pn, xbuf, (size_t)n * xs);
    s = c->stream[0];
    err = ensure_dbuf(c, xb + ALIGN16(ub));
    dx = (uint8_t *)c->dbuf[0];
    du = dx + xb;
    if (!err) err = pncxrt_memset(c->dstatus, 0, sizeof(int), s);
    if (!err) err = pncxrt_memcpy_h2d(du, ubase, ub, s);       /* user span (get: keeps the holes) */
    if (dir == PNCX_PUT) {
        if (!err && op.c) err = pncxrt_memcpy_h2d(dx, xbuf, (size_t)n * xs, s);
        if (!err) err = launch_imap_op(&op, du - lo + koff, dx, n, &m, 1, c->dstatus, s);
        if (!err) err = pncxrt_memcpy_d2h(xbuf, dx, (size_t)n * xs, s);
    } else {
        if (!err) err = pncxrt_memcpy_h2d(dx, xbuf, (size_t)n * xs, s);
        if (!err) err = launch_imap_op(&op, dx, du - lo + koff, n, &m, 0, c->dstatus, s);
        if (!err) err = pncxrt_memcpy_d2h(ubase, du, ub, s);
    }
    if (!err) err = pncxrt_memcpy_d2h(&st, c->dstatus, sizeof(int), s);
    if (!err) err = pncxrt_stream_sync(s);
    unpin_all(&pn);
    pthread_mutex_unlock(&c->lock);
    if (err) return err < 0 ? err : PNCX_EDEVICE;
    return st;
}

int pncx_putn_flex(int cdf_ver, int xtype, void *xbuf, const void *buf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                   const pncx_dtype *bt, const void *fillp)
{
    return host_flex(PNCX_PUT, cdf_ver, xtype, xbuf, (void *)buf, ndims, count, imap, bufcount, bt, fillp);
}

int pncx_getn_flex(int cdf_ver, int xtype, const void *xbuf, void *buf, int ndims,
                   const pncx_offset *count, const pncx_offset *imap, pncx_offset bufcount,
                   const pncx_dtype *bt)
{
    return host_flex(PNCX_GET, cdf_ver, xtype, (void *)xbuf, buf, ndims, count, imap, bufcount, bt, NULL);
}

/* ------------------------------------------------------------------------ */
/* batched                                                                   */
/* ------------------------------------------------------------------------ */
typedef struct bitem_t {
    op_t        op;
    int         idx;       /* index into the caller's segs */
    const void *src;
    void       *dst;
    long long   n;
} bitem_t;

static int mixable(const op_t *o)
{
    return o->kind == PNCXK_SWAP && (o->a == 1 || o->a == 2 || o->a == 4 || o->a == 8);
}

/* order: mixable same-type swaps first (one class), then by conversion class */
static int cmp_item(const void *pa, const void *pb)
{
    const bitem_t *a = (const bitem_t *)pa, *b = (const bitem_t *)pb;
    const int ma = mixable(&a->op), mb = mixable(&b->op);
    if (ma != mb) return mb - ma;
    if (!ma) {
        if (a->op.kind != b->op.kind) return a->op.kind - b->op.kind;
        if (a->op.a != b->op.a) return a->op.a - b->op.a;
        if (a->op.b != b->op.b) return a->op.b - b->op.b;
        if (a->op.c != b->op.c) return a->op.c - b->op.c;
    }
    return a->idx - b->idx;
}

/* elements before both pointers are aligned: to a 128-byte line when one
 * head reaches it for both, else the widest of 64/32/16 bytes (vec_head) */
static long long seg_head(const void *src, const void *dst, int ss, int ds, long long n)
{
    const uintptr_t s = (uintptr_t)src, d = (uintptr_t)dst;
    uintptr_t al;
    long long h;
    for (al = 128; al >= 16; al >>= 1)
        for (h = 0; h < 128 && h <= n; h++)
            if (((s + (uintptr_t)h * ss) & (al - 1)) == 0 && ((d + (uintptr_t)h * ds) & (al - 1)) == 0) return h;
    return -1;
}

/*
 * Batched launch of device-buffer segments.
 *   plan:  classify, group by conversion class (qsort), and for each class
 *          lay out one tile descriptor per segment (16B-aligned body, scalar
 *          head/remainder) with a running block offset;
 *   run:   one async upload of all descriptors (pinned mirror), a block->
 *          segment table built on the device for classes whose segments
 *          differ in size (equal sizes need none), then the class kernels
 *          back to back; statuses come back with one copy and one sync.
 */
typedef struct cls_t {
    int first, count;       /* descriptor range                       */
    long long nblocks;      /* grid of the class kernel               */
    long long uniform;      /* blocks per segment when all are equal  */
    long long map_off;      /* offset (ints) of its map in the map area, -1: none */
    pncxk_groups grp;       /* runs of equal-size segments (grp.n > 0: no map) */
    op_t op;
} cls_t;

/* segments of a class ordered by size, so equal sizes form runs */
static int cmp_seg_size(const void *pa, const void *pb)
{
    const pncxk_seg *a = (const pncxk_seg *)pa, *b = (const pncxk_seg *)pb;
    const long long na = a->nvec > 0 ? a->nvec : 1, nb = b->nvec > 0 ? b->nvec : 1;
    if (na != nb) return na < nb ? -1 : 1;
    return a->block0 < b->block0 ? -1 : a->block0 > b->block0;   /* keep plan order */
}

/* run k of a group table divides by per[k] with a multiply and a shift
 * (pncx_shim.h): shr = 31 + ceil(log2 per), mag = ceil(2^shr / per) */
static void group_magic(pncxk_groups *g, int k)
{
    const long long d = g->r[k].per;
    int l = 0;
    while ((1LL << l) < d) l++;
    g->r[k].shr = 31 + l;
    g->r[k].mag = ((1ULL << g->r[k].shr) - 1) / (unsigned long long)d + 1;
}

/* Non-uniform class: sort its segments by block count and describe the runs
 * of equal counts (at most PNCXK_MAXGRP) -- O(1) block->segment in the
 * kernel without a map kernel.  Returns 0 when there are too many sizes. */
static int make_groups(pncxk_seg *seg, int count, pncxk_groups *g)
{
    int k, n = 0;
    long long b0 = 0;
    qsort(seg, (size_t)count, sizeof *seg, cmp_seg_size);
    for (k = 0; k < count; k++) {
        const long long nb = seg[k].nvec > 0 ? seg[k].nvec : 1;
        if (n == 0 || g->r[n - 1].per != nb) {
            if (n == PNCXK_MAXGRP) return 0;
            g->r[n].s0 = k;
            g->r[n].b0 = b0;
            g->r[n].per = nb;
            n++;
        }
        seg[k].block0 = b0;
        b0 += nb;
    }
    g->n = n;
    for (k = 0; k < n; k++) group_magic(g, k);
    return 1;
}

typedef struct plan_t {
    bitem_t   *it;
    int        nit;
    pncxk_seg *seg;         /* host descriptors (later copied to the pinned mirror) */
    int        nsegd;
    cls_t     *cls;
    int        ncls;
    long long  map_ints;    /* total block-map ints */
} plan_t;

static void plan_free(plan_t *p)
{
    free(p->seg);
    free(p->cls);
    p->seg = NULL;
    p->cls = NULL;
}

static int batch_plan(plan_t *p)
{
    int i = 0, err = 0, k;
    bitem_t *it = p->it;
    const int nit = p->nit;
    p->seg = (pncxk_seg *)malloc(sizeof(pncxk_seg) * (size_t)(nit > 0 ? nit : 1));
    p->cls = (cls_t *)malloc(sizeof(cls_t) * (size_t)(nit > 0 ? nit : 1));
    p->nsegd = p->ncls = 0;
    p->map_ints = 0;
    if (p->seg == NULL || p->cls == NULL) return NC_ENOMEM;
    qsort(it, (size_t)nit, sizeof *it, cmp_item);
    while (!err && i < nit) {
        int j = i, mix;
        pncxk_opinfo oi;
        const op_t *op = &it[i].op;
        cls_t *c;
        /* all same-type swaps/copies of 1/2/4/8 bytes form ONE class (one
         * launch); other classes are one (kind, xtype, itype) each */
        mix = mixable(op);
        while (j < nit && (mix ? mixable(&it[j].op)
                               : (it[j].op.kind == op->kind && it[j].op.a == op->a &&
                                  it[j].op.b == op->b && it[j].op.c == op->c)))
            j++;
        if ((op->kind == PNCXK_SWAP && !mix) || op->c) {
            i = j;          /* generic n-byte swaps / NULL-fill codecs: run one by one */
            continue;
        }
        c = &p->cls[p->ncls];
        c->first = p->nsegd;
        c->nblocks = 0;
        c->uniform = -1;
        c->op = *op;
        if (mix) c->op.kind = PNCXK_SWAPMIX;
        for (k = i; k < j && !err; k++) {
            pncxk_seg *sg;
            long long nb, h;
            if ((err = pncxk_opinfo_get(it[k].op.kind, it[k].op.a, it[k].op.b, it[k].op.c, &oi)) != 0) break;
            h = seg_head(it[k].src, it[k].dst, oi.ss, oi.ds, it[k].n);
            if (it[k].n <= 0 || h < 0) continue;       /* empty / scalar-only: run alone */
            if (mix && it[k].src == it[k].dst && it[k].op.a == 1) { it[k].n = -it[k].n - 1; continue; }
            sg = &p->seg[p->nsegd++];
            sg->src = it[k].src;
            sg->dst = it[k].dst;
            sg->n = it[k].n;
            sg->head = h;
            /* full block tiles (the mix kernel's tile is PNCXK_MIX_LANES x 16 B) */
            sg->nvec = (it[k].n - h) / (mix ? PNCXK_MIX_LANES * 16 / it[k].op.a : oi.vec);
            sg->block0 = c->nblocks;
            sg->fill = it[k].op.fill;
            sg->status = (int *)(intptr_t)it[k].idx;     /* caller's index; pointer set at run time */
            sg->aux = it[k].op.a;
            it[k].n = -it[k].n - 1;                      /* mark as batched */
            nb = sg->nvec > 0 ? sg->nvec : 1;
            if (c->uniform == -1) c->uniform = nb;
            else if (c->uniform != nb) c->uniform = 0;
            c->nblocks += nb;
        }
        c->count = p->nsegd - c->first;
        memset(&c->grp, 0, sizeof c->grp);
        if (c->count > 0) {
            if (c->uniform > 0) {                  /* all equal: one run */
                c->grp.n = 1;
                c->grp.r[0].per = c->uniform;
                group_magic(&c->grp, 0);
                c->map_off = -1;
            } else if (make_groups(p->seg + c->first, c->count, &c->grp)) {
                c->uniform = 0;                    /* a few sizes: group table */
                c->map_off = -1;
            } else {
                int k;                             /* many sizes: device map */
                long long b0 = 0;
                c->uniform = 0;
                memset(&c->grp, 0, sizeof c->grp);
                for (k = c->first; k < c->first + c->count; k++) {   /* sorted: recompute block0 */
                    p->seg[k].block0 = b0;
                    b0 += p->seg[k].nvec > 0 ? p->seg[k].nvec : 1;
                }
                c->map_off = p->map_ints;
                p->map_ints += c->nblocks;
            }
            p->ncls++;
        }
        i = j;
    }
    return err;
}

/* scratch layout (device and pinned mirror): [statuses | descriptors | maps].
 * ONE upload zeroes the statuses and installs the descriptors; then the
 * unbatched items and the class kernels run; one copy brings the statuses back. */
/* pncx_dev_batch_timing: the event pairs are read when NTEV are in use or
 * when pncx_dev_batch_kernel_ms asks (reading them per call would add a
 * synchronize and an elapsed-time query to every timed call) */
static void batch_time_drain(ctx_t *c)
{
    int k;
    for (k = 0; k < c->tpend; k++) {
        float ms = 0.0f;
        if (pncxrt_event_sync(c->tev[2 * k + 1]) == 0 &&
            pncxrt_event_elapsed_ms(&ms, c->tev[2 * k], c->tev[2 * k + 1]) == 0)
            c->tms += ms;
    }
    c->tcalls += c->tcpend;
    c->tpend = c->tcpend = 0;
}

/* the call whose launches used the c->tnext pairs after tpend has completed
 * (tnext < 0: a call with more classes than the ring holds, not timed) */
static void batch_time(ctx_t *c)
{
    if (c->tnext < 0) {
        c->tnext = 0;
        return;
    }
    c->tpend += c->tnext;
    c->tnext = 0;
    c->tcpend++;
}

/* PNCX_BATCH_FUSE=1 runs a conversion class and the same-type swaps of one
 * batch as one launch (k_batch_fused).  Off by default: on C4's NC_ERANGE
 * variant the fused launch took 0.3026-0.3032 ms with 256-lane blocks and
 * 0.3160-0.3169 ms with 1024-lane blocks against 0.2995-0.3007 ms for the
 * two class kernels, in alternating runs on one box
 * (profiles/r03_fuse_ab.txt): the ramp and drain it saves are not where
 * the time goes.  Read per call, so tests can run both ways in one process. */
static int batch_fuse_enabled(void) { return pncx_knob(PNCXK_KNOB_BATCH_FUSE) == 1; }

/* launch the class kernels of a plan whose descriptors are on the device */
static int launch_classes(const cls_t *cls, int ncls, uint8_t *dbase, size_t soff, size_t moff, int sval,
                          int build_maps, void *stream, ctx_t *tc)
{
    int k, err = 0;
    /* timing: every class kernel's start and end are stamped by its own
     * dispatch (hipExtLaunchKernel), and a call's kernel time is the sum of
     * those intervals, as rocprof's per-kernel durations add up.  Events
     * recorded ahead of a kernel on an idle stream would also time the host's
     * launch call, and a stamped kernel delays the next one on its stream by
     * ~5 us, so an interval from the first kernel's start to the last one's
     * end would count that gap too.  The flag reduce (k_flags_*) is not
     * timed.  A call with more classes than the event ring holds goes untimed. */
    const int timed = tc != NULL && tc->timing && ncls <= NTEV;
    if (timed && tc->tpend + ncls > NTEV) batch_time_drain(tc);
    if (tc != NULL) tc->tnext = tc->timing && !timed ? -1 : 0;
    pncxk_seg *dseg = (pncxk_seg *)(dbase + soff);
    int *dmap = (int *)(dbase + moff);
    /* a conversion class beside the same-type swaps (C4's NC_ERANGE variant:
     * float -> NC_SHORT + the NC_FLOAT swaps): one fused launch
     * (k_batch_fused), one ramp and drain instead of two */
    if (ncls == 2 && batch_fuse_enabled()) {
        const int mi = cls[0].op.kind == PNCXK_SWAPMIX ? 0 : cls[1].op.kind == PNCXK_SWAPMIX ? 1 : -1;
        const cls_t *cv = mi >= 0 ? &cls[1 - mi] : NULL, *mx = mi >= 0 ? &cls[mi] : NULL;
        if (cv != NULL && (cv->op.kind == PNCXK_GET || cv->op.kind == PNCXK_PUT)) {
            pncxk_batch_args ba[2];
            const cls_t *cc[2] = {cv, mx};
            int j, rc;
            for (j = 0; j < 2; j++) {
                ba[j].dsegs = dseg + cc[j]->first;
                ba[j].nseg = cc[j]->count;
                ba[j].nblocks = cc[j]->nblocks;
                ba[j].dmap = cc[j]->map_off >= 0 ? dmap + cc[j]->map_off : NULL;
                ba[j].grp = cc[j]->grp;
                ba[j].sval = sval;
                ba[j].stream = stream;
                ba[j].ev_start = ba[j].ev_stop = NULL;
                if (ba[j].dmap != NULL && build_maps && (err = pncxk_batch_map(&ba[j])) != 0) return err;
            }
            if (timed) {
                ba[0].ev_start = tc->tev[2 * tc->tpend];
                ba[0].ev_stop = tc->tev[2 * tc->tpend + 1];
            }
            rc = pncxk_batch_fused(cv->op.kind, cv->op.a, cv->op.b, cv->op.c, &ba[0], &ba[1]);
            if (rc != PNCXK_NOFUSE) {
                if (!rc && timed) tc->tnext = 1;
                return rc;
            }
        }
    }
    for (k = 0; k < ncls && !err; k++) {
        const cls_t *c = &cls[k];
        pncxk_batch_args ba;
        ba.dsegs = dseg + c->first;
        ba.nseg = c->count;
        ba.nblocks = c->nblocks;
        ba.dmap = c->map_off >= 0 ? dmap + c->map_off : NULL;
        ba.grp = c->grp;
        ba.sval = sval;
        ba.stream = stream;
        ba.ev_start = ba.ev_stop = NULL;
        if (ba.dmap != NULL && build_maps) err = pncxk_batch_map(&ba);
        if (timed) {
            ba.ev_start = tc->tev[2 * (tc->tpend + k)];
            ba.ev_stop = tc->tev[2 * (tc->tpend + k) + 1];
        }
        if (!err) err = pncxk_batch(c->op.kind, c->op.a, c->op.b, c->op.c, &ba);
        if (!err && timed) tc->tnext = k + 1;
    }
    return err;
}

static int batch_run(plan_t *p, int nseg, uint8_t *dbase, uint8_t *hbase, size_t soff, size_t moff,
                     int sval, void *stream, ctx_t *tc, int *dstat)
{
    int k, err = 0;
    pncxk_seg *hseg = (pncxk_seg *)(hbase + soff);
    memset(hbase, 0, soff);
    for (k = 0; k < p->nsegd; k++) {
        hseg[k] = p->seg[k];
        hseg[k].status = dstat + (intptr_t)p->seg[k].status;
    }
    err = pncxrt_memcpy_h2d(dbase, hbase, soff + sizeof(pncxk_seg) * (size_t)p->nsegd, stream);
    (void)nseg;
    /* items that are not in a class: one launch each */
    for (k = 0; k < p->nit && !err; k++) {
        bitem_t *b = &p->it[k];
        if (b->n < 0) { b->n = -b->n - 1; continue; }        /* batched: restore */
        if (b->n == 0) continue;
        if (b->op.kind == PNCXK_SWAP && b->op.a == 1 && b->src == b->dst) continue;
        err = launch_op(&b->op, b->src, b->dst, b->n, dstat + b->idx, stream);
    }
    if (!err) err = launch_classes(p->cls, p->ncls, dbase, soff, moff, sval, 1, stream, tc);
    return err;
}

/* Completion of a synchronous batch: one block copies the n status words
 * into host-mapped memory and then sets the completion word, which the host
 * polls for up to 20 ms before it blocks on the stream.  Returns with the
 * statuses at c->hdone_h + 16. */
static int done_wait(ctx_t *c, const int *dstat, int n, void *stream)
{
    struct timespec t0, t;
    int seq, err;
    if (c->hdone_cap < n || c->hdone_h == NULL) {
        void *h, *d;
        const int cap = n < 1024 ? 1024 : 2 * n;
        pncxrt_host_free(c->hdone_h);         /* no completion kernel is outstanding */
        c->hdone_h = c->hdone_d = NULL;
        c->hdone_cap = 0;
        if (pncxrt_host_alloc_mapped(&h, &d, sizeof(int) * (size_t)(16 + cap)) != 0) return PNCX_EDEVICE;
        c->hdone_h = (int *)h;
        c->hdone_d = (int *)d;
        c->hdone_cap = cap;
        __atomic_store_n(c->hdone_h, 0, __ATOMIC_RELEASE);
    }
    seq = c->done_seq = (c->done_seq + 1) & 0x7fffffff;
    if (seq == 0) seq = c->done_seq = 1;
    if ((err = pncxk_batch_done(dstat, n, c->hdone_d + 16, c->hdone_d, seq, stream)) != 0) return err;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (;;) {
        if (__atomic_load_n(c->hdone_h, __ATOMIC_ACQUIRE) == seq) return 0;
        clock_gettime(CLOCK_MONOTONIC, &t);
        if ((t.tv_sec - t0.tv_sec) * 1000000000LL + (t.tv_nsec - t0.tv_nsec) > 20000000LL) break;
    }
    if ((err = pncxrt_stream_sync(stream)) != 0) return err;
    return __atomic_load_n(c->hdone_h, __ATOMIC_ACQUIRE) == seq ? 0 : PNCX_EDEVICE;
}

/* the fill value a put segment's plan was classified with (classify copies
 * xlen bytes of *fillp into the op), zero-extended; 0 for gets and NULL fills */
static uint64_t fill_word(const pncx_seg *s)
{
    uint64_t w = 0;
    const int xs = pncx_xlen(s->xtype);
    if (s->dir == PNCX_PUT && s->fillp != NULL && xs > 0 && xs <= 8) memcpy(&w, s->fillp, (size_t)xs);
    return w;
}

static int same_fills(const uint64_t *cached, const pncx_seg *segs, int nseg)
{
    int i;
    for (i = 0; i < nseg; i++)
        if (cached[i] != fill_word(&segs[i])) return 0;
    return 1;
}

/* dstatus == NULL: synchronous pncx_dev_batch (statuses come back to the
 * host, epoch values in the scratch status words); else pncx_dev_batch_async
 * (the kernels set the caller's device words to NC_ERANGE; nothing waits) */
static int dev_batch(const pncx_seg *segs, int nseg, int *status_out, int *dstatus, pncx_stream_t stream)
{
    ctx_t *c;
    plan_t plan;
    int *hstat, i, err = 0, first = NC_NOERR, sval, nclassified = 0, unbatched = 0, swaponly = 1;
    const int async = dstatus != NULL;
    if (nseg <= 0) return NC_NOERR;
    if (segs == NULL) return NC_EINVAL;
    if (!have_device()) return PNCX_EDEVICE;
    c = get_ctx();
    if (c == NULL) return PNCX_EDEVICE;
    hstat = (int *)calloc((size_t)nseg, sizeof(int));
    if (hstat == NULL) return NC_ENOMEM;
    pthread_mutex_lock(&c->lock);
    /* batch kernels write sval (this call's epoch) on ERANGE: old words can
     * stay in place, so a repeated segment list needs no upload at all */
    c->epoch = (c->epoch + 1) & 0x3fffffff;
    if (c->epoch == 0) { c->epoch = 1; c->cache_valid = 0; }
    sval = async ? NC_ERANGE : 0x40000000 | c->epoch;
    if (c->cache_valid && c->cache_nseg == nseg && c->cache_dstatus == dstatus &&
        memcmp(c->cache_segs, segs, sizeof(pncx_seg) * (size_t)nseg) == 0 &&
        same_fills(c->cache_fills, segs, nseg)) {
        /* async calls on a cached plan read the device descriptors until they
         * finish: the next re-plan waits for their stream, so only one stream
         * may have such calls outstanding -- switching streams drains the old one */
        if (async && c->async_pending && c->async_stream != stream) err = pncxrt_stream_sync(c->async_stream);
        if (!err)
            err = launch_classes(c->cache_cls, c->cache_ncls, (uint8_t *)c->dscratch, c->cache_soff,
                                 c->cache_moff, sval, 0, stream, c);
        if (async && !err) {
            c->async_pending = 1;
            c->async_stream = stream;
            if (c->timing) batch_time(c);       /* events read at the next drain */
        }
        if (!async) {
            /* byte swaps and copies never raise NC_ERANGE: no statuses to bring back */
            if (!err) err = done_wait(c, (const int *)c->dscratch, c->cache_swaponly ? 0 : nseg, stream);
            if (!err && c->timing) batch_time(c);
            if (!err)
                for (i = 0; i < nseg; i++)
                    hstat[i] = !c->cache_swaponly && c->hdone_h[16 + i] == sval ? NC_ERANGE : NC_NOERR;
        }
        pthread_mutex_unlock(&c->lock);
        goto out;
    }
    /* a new plan rewrites the pinned mirror and the device descriptors: an
     * async call's upload (or its kernels) may still be reading them */
    if (c->async_pending) {
        err = pncxrt_stream_sync(c->async_stream);
        c->async_pending = 0;
        if (err) { pthread_mutex_unlock(&c->lock); free(hstat); return PNCX_EDEVICE; }
    }
    memset(&plan, 0, sizeof plan);
    plan.it = (bitem_t *)calloc((size_t)nseg, sizeof *plan.it);
    if (plan.it == NULL) { pthread_mutex_unlock(&c->lock); free(hstat); return NC_ENOMEM; }
    for (i = 0; i < nseg; i++) {
        const pncx_seg *sg = &segs[i];
        bitem_t *bi = &plan.it[plan.nit];
        int e = classify(sg->dir, sg->cdf_ver, sg->xtype, sg->itype, sg->fillp, &bi->op);
        if (e != NC_NOERR) { hstat[i] = e; continue; }
        bi->idx = i;
        bi->n = sg->nelems > 0 ? sg->nelems : 0;
        bi->src = sg->dir == PNCX_PUT ? sg->ibuf : sg->xbuf;
        bi->dst = sg->dir == PNCX_PUT ? sg->xbuf : sg->ibuf;
        plan.nit++;
        nclassified++;
    }
    for (i = 0; i < plan.nit; i++)
        if (plan.it[i].op.kind != PNCXK_SWAP) swaponly = 0;
    err = batch_plan(&plan);
    for (i = 0; i < plan.nit; i++) {       /* items a class kernel does not cover run alone */
        const bitem_t *bi = &plan.it[i];
        if (bi->n > 0 && !(bi->op.kind == PNCXK_SWAP && bi->op.a == 1 && bi->src == bi->dst)) unbatched++;
    }
    if (!err) {
        /* scratch layout: [statuses | descriptors | block maps] */
        const size_t soff = ALIGN16(sizeof(int) * (size_t)nseg);
        const size_t moff = soff + ALIGN16(sizeof(pncxk_seg) * (size_t)(plan.nsegd + 1));
        err = ensure_scratch(c, moff + sizeof(int) * (size_t)plan.map_ints + 16);
        if (!err)
            err = batch_run(&plan, nseg, (uint8_t *)c->dscratch, (uint8_t *)c->hscratch, soff, moff, sval, stream,
                            c, async ? dstatus : (int *)c->dscratch);
        if (async) {
            if (!err) { c->async_pending = 1; c->async_stream = stream; }
            if (!err && c->timing) batch_time(c);
        } else {
            /* the status words were zeroed by the upload; a batch of swaps
             * and copies only has nothing to read */
            if (!err) err = done_wait(c, (const int *)c->dscratch, swaponly ? 0 : nseg, stream);
            if (!err && c->timing) batch_time(c);
            if (!err && !swaponly)
                for (i = 0; i < nseg; i++)
                    if (hstat[i] == NC_NOERR) hstat[i] = c->hdone_h[16 + i] != 0 ? NC_ERANGE : NC_NOERR;
        }
        /* keep the plan when every segment runs in a class kernel */
        c->cache_valid = 0;
        if (!err && unbatched == 0 && nclassified == nseg) {
            pncx_seg *cs = (pncx_seg *)realloc(c->cache_segs, sizeof(pncx_seg) * (size_t)nseg);
            cls_t *cc = (cls_t *)realloc(c->cache_cls, sizeof(cls_t) * (size_t)(plan.ncls ? plan.ncls : 1));
            uint64_t *cf = (uint64_t *)realloc(c->cache_fills, sizeof(uint64_t) * (size_t)nseg);
            if (cs) c->cache_segs = cs;
            if (cc) c->cache_cls = cc;
            if (cf) c->cache_fills = cf;
            if (cs && cc && cf) {
                memcpy(cs, segs, sizeof(pncx_seg) * (size_t)nseg);
                for (i = 0; i < nseg; i++) cf[i] = fill_word(&segs[i]);
                memcpy(cc, plan.cls, sizeof(cls_t) * (size_t)plan.ncls);
                c->cache_nseg = nseg;
                c->cache_ncls = plan.ncls;
                c->cache_swaponly = swaponly;
                c->cache_dstatus = dstatus;
                c->cache_soff = soff;
                c->cache_moff = moff;
                c->cache_valid = 1;
            }
        }
    }
    pthread_mutex_unlock(&c->lock);
    plan_free(&plan);
    free(plan.it);
out:
    if (!err)
        for (i = 0; i < nseg; i++) {
            if (status_out) status_out[i] = hstat[i];
            if (first == NC_NOERR) first = hstat[i];
        }
    free(hstat);
    return err ? (err < 0 ? err : PNCX_EDEVICE) : first;
}

int pncx_dev_batch(const pncx_seg *segs, int nseg, int *status_out, pncx_stream_t stream)
{
    return dev_batch(segs, nseg, status_out, NULL, stream);
}

int pncx_dev_batch_async(const pncx_seg *segs, int nseg, int *dstatus, pncx_stream_t stream)
{
    if (dstatus == NULL && nseg > 0) return NC_EINVAL;
    return dev_batch(segs, nseg, NULL, dstatus, stream);
}

int pncx_dev_batch_timing(int enable)
{
    ctx_t *c;
    if (!have_device() || (c = get_ctx()) == NULL) return PNCX_EDEVICE;
    pthread_mutex_lock(&c->lock);
    if (enable && c->tev[2 * NTEV - 1] == NULL) {
        int k;
        for (k = 0; k < 2 * NTEV; k++)
            if (c->tev[k] == NULL && pncxrt_event_create(&c->tev[k]) != 0) {
                c->tev[k] = NULL;
                pthread_mutex_unlock(&c->lock);
                return PNCX_EDEVICE;
            }
    }
    c->timing = enable != 0;
    c->tpend = c->tcpend = c->tnext = 0;
    c->tms = 0.0;
    c->tcalls = 0;
    pthread_mutex_unlock(&c->lock);
    return NC_NOERR;
}

int pncx_dev_batch_kernel_ms(double *total_ms, long long *calls)
{
    ctx_t *c;
    if (total_ms == NULL || calls == NULL) return NC_EINVAL;
    *total_ms = 0.0;
    *calls = 0;
    if (!have_device() || (c = get_ctx()) == NULL) return PNCX_EDEVICE;
    pthread_mutex_lock(&c->lock);
    batch_time_drain(c);
    *total_ms = c->tms;
    *calls = c->tcalls;
    pthread_mutex_unlock(&c->lock);
    return NC_NOERR;
}

/* Zero-copy batch: every segment's host buffers are pinned or registered
 * for the call, and the batch kernels load from and store to them over PCIe
 * in one pass (a staged batch copies everything up, converts, copies
 * everything back).  Returns 1 when it ran (*ret set), 0 when some buffer
 * could not be mapped (nothing was launched; the caller stages). */
static int batch_zero_copy(const pncx_seg *segs, int nseg, int *status_out, void *stream, int *ret)
{
    pncx_seg *zs = (pncx_seg *)calloc((size_t)nseg, sizeof *zs);
    void **reg = (void **)calloc((size_t)(2 * nseg), sizeof(void *));
    int i, nreg = 0, ok = zs != NULL && reg != NULL;
    for (i = 0; i < nseg && ok; i++) {
        const pncx_seg *s = &segs[i];
        const int xs = pncx_xlen(s->xtype), is = pncx_ilen(s->itype);
        int side;
        zs[i] = *s;
        if (xs < 0 || is < 0 || s->nelems <= 0) continue;       /* dev_batch reports these */
        for (side = 0; side < 2 && ok; side++) {
            void *h = side ? s->ibuf : s->xbuf;
            const size_t nb = (size_t)s->nelems * (size_t)(side ? is : xs);
            void *d = pncxrt_host_dptr_range(h, nb);
            if (d == NULL) {
                const int r = pncxrt_host_register(h, nb);
                if (r == 0) reg[nreg++] = h;
                d = r >= 0 ? pncxrt_host_dptr_range(h, nb) : NULL;
            }
            if (d == NULL) ok = 0;
            else if (side) zs[i].ibuf = d;
            else zs[i].xbuf = d;
        }
    }
    if (ok) *ret = pncx_dev_batch(zs, nseg, status_out, stream);
    for (i = 0; i < nreg; i++) pncxrt_host_unregister(reg[i]);
    free(zs);
    free(reg);
    return ok;
}

int pncx_batch(const pncx_seg *segs, int nseg, int *status_out)
{
    /* Zero copy where every buffer can be mapped (PNCX_HOST_ZC >= 2, the
     * default); else stage every segment into one device arena (16B-aligned
     * slots), run the device batch, copy the outputs back. */
    ctx_t *c;
    pncx_seg *dsegs = NULL;
    size_t total = 0, off = 0;
    int i, err = 0, ret;
    uint8_t *arena = NULL;
    if (nseg <= 0) return NC_NOERR;
    if (segs == NULL) return NC_EINVAL;
    if (!have_device()) return PNCX_EDEVICE;
    c = get_ctx();
    if (c == NULL) return PNCX_EDEVICE;
    {
        long long bytes = 0;
        for (i = 0; i < nseg; i++) {
            const int xs = pncx_xlen(segs[i].xtype), is = pncx_ilen(segs[i].itype);
            if (xs > 0 && is > 0 && segs[i].nelems > 0) bytes += segs[i].nelems * (long long)(xs + is);
        }
        if (stage_mode(bytes) == STAGE_ZC && batch_zero_copy(segs, nseg, status_out, c->stream[0], &ret)) return ret;
    }
    dsegs = (pncx_seg *)calloc((size_t)nseg, sizeof *dsegs);
    if (dsegs == NULL) return NC_ENOMEM;
    for (i = 0; i < nseg; i++) {
        const int xs = pncx_xlen(segs[i].xtype), is = pncx_ilen(segs[i].itype);
        if (xs < 0 || is < 0 || segs[i].nelems <= 0) continue;
        total += ALIGN16((size_t)segs[i].nelems * xs) + ALIGN16((size_t)segs[i].nelems * is);
    }
    if (total == 0) total = 16;
    pthread_mutex_lock(&c->block);
    if (c->barena_size < total) {           /* grow-only: hipMalloc per call costs more than the batch */
        if (c->barena) pncxrt_free(c->barena);
        c->barena = NULL;
        c->barena_size = 0;
        if (pncxrt_malloc(&c->barena, total) != 0) {
            pthread_mutex_unlock(&c->block);
            free(dsegs);
            return PNCX_EDEVICE;
        }
        c->barena_size = total;
    }
    arena = (uint8_t *)c->barena;
    for (i = 0; i < nseg && !err; i++) {
        const pncx_seg *s = &segs[i];
        const int xs = pncx_xlen(s->xtype), is = pncx_ilen(s->itype);
        dsegs[i] = *s;
        if (xs < 0 || is < 0 || s->nelems <= 0) continue;
        dsegs[i].xbuf = arena + off;
        off += ALIGN16((size_t)s->nelems * xs);
        dsegs[i].ibuf = arena + off;
        off += ALIGN16((size_t)s->nelems * is);
        if (s->dir == PNCX_PUT) {
            err = pncxrt_memcpy_h2d(dsegs[i].ibuf, s->ibuf, (size_t)s->nelems * is, c->stream[0]);
            if (!err && s->fillp == NULL)   /* NULL-fill codecs read xbuf */
                err = pncxrt_memcpy_h2d(dsegs[i].xbuf, s->xbuf, (size_t)s->nelems * xs, c->stream[0]);
        } else {
            err = pncxrt_memcpy_h2d(dsegs[i].xbuf, s->xbuf, (size_t)s->nelems * xs, c->stream[0]);
        }
    }
    ret = err ? PNCX_EDEVICE : pncx_dev_batch(dsegs, nseg, status_out, c->stream[0]);
    for (i = 0; i < nseg && !err; i++) {
        const pncx_seg *s = &segs[i];
        const int xs = pncx_xlen(s->xtype), is = pncx_ilen(s->itype);
        if (xs < 0 || is < 0 || s->nelems <= 0) continue;
        if (s->dir == PNCX_PUT)
            err = pncxrt_memcpy_d2h(s->xbuf, dsegs[i].xbuf, (size_t)s->nelems * xs, c->stream[0]);
        else
            err = pncxrt_memcpy_d2h(s->ibuf, dsegs[i].ibuf, (size_t)s->nelems * is, c->stream[0]);
    }
    if (!err) err = pncxrt_stream_sync(c->stream[0]);
    pthread_mutex_unlock(&c->block);
    free(dsegs);
    if (err) return PNCX_EDEVICE;
    return ret;
}
