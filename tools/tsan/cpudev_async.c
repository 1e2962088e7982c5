/*
 * An ASYNCHRONOUS CPU stand-in for the HIP shim (pncx_shim.h), used ONLY by
 * test builds on a machine without a GPU (tools/tsan/run_async.sh, the
 * file-layer fuzz on CPU).  Never linked into the library.
 *
 * tools/tsan/cpudev_stub.c runs every device operation at once on the
 * calling thread, so a missing wait in the host code cannot show there.
 * Here each stream is a FIFO worker thread: copies, memsets and kernels are
 * queued and run later, events complete when their stream reaches them,
 * stream waits order one worker behind another, and the batch completion
 * word is set by the worker -- the host code's synchronisation is exercised
 * the way the GPU exercises it, and under ThreadSanitizer every host access
 * that is not ordered after the "device" access it depends on is reported.
 *
 * The conversions themselves are the CPU oracle's (oracle/pncx_oracle.c,
 * test infrastructure): putn / getn per launch and per batch segment,
 * NC_ERANGE into the status word (launch) or the batch's status value (sval).
 * The varm / flexible gather kernels are not emulated (no device).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../pnetcdf_amd/csrc/pncx_shim.h"

#define NODEV (-1900)
#define ERANGE_ (-60)

int orc_getn(int cdf_ver, int xtype, const void *xbuf, void *ibuf, long long nelems, int itype);
int orc_putn(int cdf_ver, int xtype, void *xbuf, const void *ibuf, long long nelems, int itype, const void *fillp);
int orc_xlen(int xtype);
int orc_ilen(int itype);

/* ------------------------------------------------------------------ streams */
typedef struct op {
    struct op *next;
    void (*fn)(struct op *);
    void *a, *b;
    size_t n;
    int i0, i1, i2, i3;
    pncxk_args args;
    pncxk_batch_args bargs;
    struct cevent *ev;
} op;

typedef struct cstream {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    op *head, *tail;
    unsigned long long enq, done;
    pthread_t th;
} cstream;

typedef struct cevent {
    cstream *s;
    unsigned long long seq;
} cevent;

static void *worker(void *arg)
{
    cstream *s = (cstream *)arg;
    for (;;) {
        op *o;
        pthread_mutex_lock(&s->mu);
        while (s->head == NULL) pthread_cond_wait(&s->cv, &s->mu);
        o = s->head;
        pthread_mutex_unlock(&s->mu);
        o->fn(o);
        pthread_mutex_lock(&s->mu);
        s->head = o->next;
        if (s->head == NULL) s->tail = NULL;
        s->done++;
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
        free(o);
    }
    return NULL;
}

static cstream *new_stream(void)
{
    cstream *s = (cstream *)calloc(1, sizeof *s);
    pthread_attr_t at;
    if (s == NULL) return NULL;
    pthread_mutex_init(&s->mu, NULL);
    pthread_cond_init(&s->cv, NULL);
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    pthread_create(&s->th, &at, worker, s);
    pthread_attr_destroy(&at);
    return s;
}

static cstream *g_null;
static pthread_once_t g_null_once = PTHREAD_ONCE_INIT;
static void null_init(void) { g_null = new_stream(); }

static cstream *S(void *s)
{
    if (s != NULL) return (cstream *)s;
    pthread_once(&g_null_once, null_init);
    return g_null;
}

static int enqueue(void *stream, op *o)
{
    cstream *s = S(stream);
    o->next = NULL;
    pthread_mutex_lock(&s->mu);
    if (s->tail) s->tail->next = o; else s->head = o;
    s->tail = o;
    s->enq++;
    pthread_cond_broadcast(&s->cv);
    pthread_mutex_unlock(&s->mu);
    return 0;
}

static op *new_op(void (*fn)(op *))
{
    op *o = (op *)calloc(1, sizeof *o);
    if (o) o->fn = fn;
    return o;
}

static void wait_seq(cstream *s, unsigned long long seq)
{
    pthread_mutex_lock(&s->mu);
    while (s->done < seq) pthread_cond_wait(&s->cv, &s->mu);
    pthread_mutex_unlock(&s->mu);
}

/* ------------------------------------------------------------------ memory */
/* every range a kernel may touch: device allocations (kind 0), pinned host
 * allocations (1) and host ranges registered for the device (2).  A kernel
 * that touches anything else at the time it RUNS aborts the program: on the
 * GPU that is an illegal address (or a write to pages the device no longer
 * maps, e.g. after an unregister that came too early). */
#define MAXALLOC 4096
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static struct { char *p; size_t n; int kind; } g_alloc[MAXALLOC];

static int add_range(void *p, size_t n, int kind)
{
    int i;
    pthread_mutex_lock(&g_mu);
    for (i = 0; i < MAXALLOC && g_alloc[i].p; i++) {}
    if (i < MAXALLOC) { g_alloc[i].p = (char *)p; g_alloc[i].n = n ? n : 1; g_alloc[i].kind = kind; }
    pthread_mutex_unlock(&g_mu);
    return i < MAXALLOC ? 0 : NODEV;
}

static void del_range(void *p, int kind)
{
    int i;
    pthread_mutex_lock(&g_mu);
    for (i = 0; i < MAXALLOC; i++)
        if (g_alloc[i].p == p && g_alloc[i].kind == kind) { g_alloc[i].p = NULL; g_alloc[i].n = 0; break; }
    pthread_mutex_unlock(&g_mu);
}

/* the entry holding [p, p + n) (kind < 0: any), or -1 */
static int find_range(const void *p, size_t n, int kind)
{
    int i, r = -1;
    const char *q = (const char *)p;
    pthread_mutex_lock(&g_mu);
    for (i = 0; i < MAXALLOC && r < 0; i++)
        if (g_alloc[i].p && (kind < 0 || g_alloc[i].kind == kind) && q >= g_alloc[i].p &&
            q + n <= g_alloc[i].p + g_alloc[i].n)
            r = i;
    pthread_mutex_unlock(&g_mu);
    return r;
}

static int find_alloc(const void *p) { return find_range(p, 1, 0); }

static void check_access(const void *p, size_t n, const char *what)
{
    if (n == 0 || find_range(p, n, -1) >= 0) return;
    fprintf(stderr, "cpudev: %s touches %p + %zu, which no device allocation, pinned or registered range "
            "covers when the kernel runs\n", what, p, n);
    abort();
}

int pncxrt_device_count(void) { return 1; }
int pncxrt_set_device(int dev) { return dev == 0 ? 0 : NODEV; }
int pncxrt_get_device(void) { return 0; }
int pncxrt_load_swap_code(void) { return 0; }
int pncxk_load_xtype(int x) { (void)x; return 0; }

int pncxrt_malloc(void **p, size_t n)
{
    char *q = (char *)malloc(n ? n : 1);
    if (q == NULL) return NODEV;
    if (add_range(q, n, 0) != 0) { free(q); return NODEV; }
    *p = q;
    return 0;
}

static void drain_all(void);

int pncxrt_free(void *p)
{
    if (p == NULL) return 0;
    drain_all();                       /* hipFree waits for the device */
    del_range(p, 0);
    free(p);
    return 0;
}

int pncxrt_host_alloc(void **p, size_t n)
{
    if ((*p = calloc(1, n ? n : 1)) == NULL) return NODEV;
    return add_range(*p, n, 1);
}
int pncxrt_host_alloc_mapped(void **p, void **dp, size_t n)
{
    if ((*p = *dp = calloc(1, n ? n : 1)) == NULL) return NODEV;
    return add_range(*p, n, 1);
}
int pncxrt_host_free(void *p)
{
    if (p == NULL) return 0;
    drain_all();
    del_range(p, 1);
    free(p);
    return 0;
}

static void do_copy(op *o) { memmove(o->a, o->b, o->n); }
static void do_set(op *o) { memset(o->a, o->i0, o->n); }

static int copy_async(void *d, const void *s, size_t n, void *stream)
{
    op *o = new_op(do_copy);
    if (o == NULL) return NODEV;
    o->a = d;
    o->b = (void *)s;
    o->n = n;
    return enqueue(stream, o);
}
int pncxrt_memcpy_h2d(void *d, const void *h, size_t n, void *s) { return copy_async(d, h, n, s); }
int pncxrt_memcpy_d2h(void *h, const void *d, size_t n, void *s) { return copy_async(h, d, n, s); }
int pncxrt_memcpy_d2d(void *d, const void *x, size_t n, void *s) { return copy_async(d, x, n, s); }
int pncxrt_memset(void *d, int v, size_t n, void *s)
{
    op *o = new_op(do_set);
    if (o == NULL) return NODEV;
    o->a = d;
    o->i0 = v;
    o->n = n;
    return enqueue(s, o);
}

/* ------------------------------------------------------------------ streams / events */
#define MAXSTREAM 256
static cstream *g_streams[MAXSTREAM];
static int g_nstreams;

int pncxrt_stream_create(void **s)
{
    cstream *c = new_stream();
    if (c == NULL) return NODEV;
    pthread_mutex_lock(&g_mu);
    if (g_nstreams < MAXSTREAM) g_streams[g_nstreams++] = c;
    pthread_mutex_unlock(&g_mu);
    *s = c;
    return 0;
}
int pncxrt_stream_destroy(void *s) { if (s) wait_seq((cstream *)s, ((cstream *)s)->enq); return 0; }

int pncxrt_stream_sync(void *s)
{
    cstream *c = S(s);
    unsigned long long target;
    pthread_mutex_lock(&c->mu);
    target = c->enq;
    pthread_mutex_unlock(&c->mu);
    wait_seq(c, target);
    return 0;
}

static void drain_all(void)
{
    int i, n;
    pthread_mutex_lock(&g_mu);
    n = g_nstreams;
    pthread_mutex_unlock(&g_mu);
    for (i = 0; i < n; i++) pncxrt_stream_sync(g_streams[i]);
    pncxrt_stream_sync(NULL);
}

int pncxrt_event_create(void **e) { return (*e = calloc(1, sizeof(cevent))) ? 0 : NODEV; }
int pncxrt_event_create_fast(void **e) { return pncxrt_event_create(e); }
int pncxrt_event_destroy(void *e) { free(e); return 0; }
int pncxrt_event_record(void *e, void *s)
{
    cevent *ev = (cevent *)e;
    cstream *c = S(s);
    pthread_mutex_lock(&c->mu);
    ev->s = c;
    ev->seq = c->enq;
    pthread_mutex_unlock(&c->mu);
    return 0;
}
static void do_wait_event(op *o) { wait_seq((cstream *)o->a, (unsigned long long)o->n); }
int pncxrt_stream_wait_event(void *s, void *e)
{
    cevent *ev = (cevent *)e;
    op *o;
    if (ev->s == NULL) return 0;
    o = new_op(do_wait_event);
    if (o == NULL) return NODEV;
    o->a = ev->s;
    o->n = (size_t)ev->seq;
    return enqueue(s, o);
}
int pncxrt_event_sync(void *e)
{
    cevent *ev = (cevent *)e;
    if (ev->s) wait_seq(ev->s, ev->seq);
    return 0;
}
int pncxrt_event_query(void *e)
{
    cevent *ev = (cevent *)e;
    int r;
    if (ev->s == NULL) return 1;
    pthread_mutex_lock(&ev->s->mu);
    r = ev->s->done >= ev->seq;
    pthread_mutex_unlock(&ev->s->mu);
    return r;
}
int pncxrt_event_elapsed_ms(float *ms, void *a, void *b) { (void)a; (void)b; *ms = 0.f; return 0; }

int pncxrt_is_device_ptr(const void *p) { return find_alloc(p) >= 0; }
int pncxrt_ptr_device(const void *p) { return find_alloc(p) >= 0 ? 0 : -1; }
/* registration as the runtime does it: an address inside a pinned or
 * registered range is already mapped (1), else the range is registered (0);
 * unregistering does NOT wait for the device (neither does
 * hipHostUnregister's contract): a kernel still queued on the range aborts */
int pncxrt_host_register(void *p, size_t n)
{
    if (find_range(p, 1, 1) >= 0 || find_range(p, 1, 2) >= 0) return 1;
    return add_range(p, n, 2) == 0 ? 0 : NODEV;
}
int pncxrt_host_unregister(void *p) { del_range(p, 2); return 0; }
void *pncxrt_host_dptr(const void *p)
{
    return find_range(p, 1, 1) >= 0 || find_range(p, 1, 2) >= 0 ? (void *)p : NULL;
}
void *pncxrt_host_dptr_range(const void *p, size_t n)
{
    return find_range(p, n ? n : 1, 1) >= 0 || find_range(p, n ? n : 1, 2) >= 0 ? (void *)p : NULL;
}
int pncxrt_host_register_map(void *p, size_t n, int r) { (void)r; return add_range(p, n, 2); }
const char *pncxrt_last_error(void) { return "asynchronous CPU stand-in"; }

/* ------------------------------------------------------------------ kernels */
static void swap_n(void *dst, const void *src, long long n, int e)
{
    unsigned char *d = (unsigned char *)dst;
    const unsigned char *s = (const unsigned char *)src;
    long long i;
    int k;
    if (e == 1) { memmove(d, s, (size_t)n); return; }
    for (i = 0; i < n; i++) {
        unsigned char t[64];
        for (k = 0; k < e; k++) t[k] = s[i * e + e - 1 - k];
        memcpy(d + i * e, t, (size_t)e);
    }
}

static void do_swap(op *o)
{
    check_access(o->args.src, (size_t)o->args.n * o->i0, "swap src");
    check_access(o->args.dst, (size_t)o->args.n * o->i0, "swap dst");
    swap_n(o->args.dst, o->args.src, o->args.n, o->i0);
}
int pncxk_swap(int e, const pncxk_args *a)
{
    op *o;
    if (e < 1 || e > 64) return NODEV;
    if ((o = new_op(do_swap)) == NULL) return NODEV;
    o->args = *a;
    o->i0 = e;
    return enqueue(a->stream, o);
}
int pncxk_swap_generic(int e, const pncxk_args *a) { return pncxk_swap(e, a); }

static void do_get(op *o)
{
    check_access(o->args.src, (size_t)o->args.n * orc_xlen(o->i0), "get src");
    check_access(o->args.dst, (size_t)o->args.n * orc_ilen(o->i1), "get dst");
    const int st = orc_getn(5, o->i0, o->args.src, o->args.dst, o->args.n, o->i1);
    if (st == ERANGE_ && o->args.status) *o->args.status = ERANGE_;
}
static void do_put(op *o)
{
    check_access(o->args.src, (size_t)o->args.n * orc_ilen(o->i1), "put src");
    check_access(o->args.dst, (size_t)o->args.n * orc_xlen(o->i0), "put dst");
    const int st = orc_putn(5, o->i0, o->args.dst, o->args.src, o->args.n, o->i1, o->i2 ? NULL : &o->args.fill);
    if (st == ERANGE_ && o->args.status) *o->args.status = ERANGE_;
}
int pncxk_get(int x, int i, const pncxk_args *a)
{
    op *o = new_op(do_get);
    if (o == NULL) return NODEV;
    o->args = *a;
    o->i0 = x;
    o->i1 = i;
    return enqueue(a->stream, o);
}
int pncxk_put(int x, int i, int p, const pncxk_args *a)
{
    op *o = new_op(do_put);
    if (o == NULL) return NODEV;
    o->args = *a;
    o->i0 = x;
    o->i1 = i;
    o->i2 = p;
    return enqueue(a->stream, o);
}

static void do_batch(op *o)
{
    const pncxk_batch_args *x = &o->bargs;
    int s;
    check_access(x->dsegs, sizeof(pncxk_seg) * (size_t)x->nseg, "batch descriptors");
    for (s = 0; s < x->nseg; s++) {
        const pncxk_seg *g = &x->dsegs[s];
        int st = 0;
        size_t sb, db;
        if (o->i0 == PNCXK_SWAP) sb = db = (size_t)g->n * o->i1;
        else if (o->i0 == PNCXK_SWAPMIX) sb = db = (size_t)g->n * g->aux;
        else if (o->i0 == PNCXK_GET) { sb = (size_t)g->n * orc_xlen(o->i1); db = (size_t)g->n * orc_ilen(o->i2); }
        else { sb = (size_t)g->n * orc_ilen(o->i2); db = (size_t)g->n * orc_xlen(o->i1); }
        check_access(g->src, sb, "batch segment src");
        check_access(g->dst, db, "batch segment dst");
        if (o->i0 == PNCXK_SWAP) swap_n(g->dst, g->src, g->n, o->i1);
        else if (o->i0 == PNCXK_SWAPMIX) swap_n(g->dst, g->src, g->n, g->aux);
        else if (o->i0 == PNCXK_GET) st = orc_getn(5, o->i1, g->src, g->dst, g->n, o->i2);
        else st = orc_putn(5, o->i1, g->dst, g->src, g->n, o->i2, o->i3 ? NULL : &g->fill);
        if (st == ERANGE_ && g->status) *g->status = x->sval;
    }
}
int pncxk_batch(int k, int a, int b, int c, const pncxk_batch_args *x)
{
    op *o = new_op(do_batch);
    if (o == NULL) return NODEV;
    o->bargs = *x;
    o->i0 = k;
    o->i1 = a;
    o->i2 = b;
    o->i3 = c;
    return enqueue(x->stream, o);
}
int pncxk_batch_fused(int k, int a, int b, int c, const pncxk_batch_args *x, const pncxk_batch_args *y)
{ (void)k; (void)a; (void)b; (void)c; (void)x; (void)y; return NODEV; }
/* varm gather (put) / scatter (get) without a derived buftype (tmode 0):
 * packed element k <-> user element sum_d idx_d(k) * imap[d] */
static long long imap_off(long long k, const pncxk_imap *m)
{
    long long off = 0;
    int d;
    for (d = m->ndims - 1; d > 0; d--) {
        off += (k % m->count[d]) * m->imap[d];
        k /= m->count[d];
    }
    return off + k * m->imap[0];
}
static void do_imap(op *o)
{
    const pncxk_imap *m = (const pncxk_imap *)o->b;
    const int kind = o->i0, a = o->i1, b = o->i2, gather = o->i3;
    const int ss = kind == PNCXK_PUT ? orc_ilen(b) : kind == PNCXK_GET ? orc_xlen(a) : a;
    const int ds = kind == PNCXK_PUT ? orc_xlen(a) : kind == PNCXK_GET ? orc_ilen(b) : a;
    const unsigned char *src = (const unsigned char *)o->args.src;
    unsigned char *dst = (unsigned char *)o->args.dst;
    long long k, jmax = 0;
    int bad = 0;
    for (k = 0; k < o->args.n; k++)
        if (imap_off(k, m) > jmax) jmax = imap_off(k, m);
    check_access(src, (size_t)(gather ? jmax + 1 : o->args.n) * ss, "imap src");
    check_access(dst, (size_t)(gather ? o->args.n : jmax + 1) * ds, "imap dst");
    for (k = 0; k < o->args.n; k++) {
        const long long j = imap_off(k, m);
        const unsigned char *sp = src + (gather ? j : k) * ss;
        unsigned char *dp = dst + (gather ? k : j) * ds;
        int st = 0;
        if (kind == PNCXK_SWAP) swap_n(dp, sp, 1, a);
        else if (kind == PNCXK_GET) st = orc_getn(5, a, sp, dp, 1, b);
        else st = orc_putn(5, a, dp, sp, 1, b, o->n ? NULL : &o->args.fill);    /* n: preserve */
        if (st == ERANGE_) bad = 1;
    }
    if (bad && o->args.status) *o->args.status = ERANGE_;
    free(o->b);
}
int pncxk_launch_imap(int k, int a, int b, int c, const pncxk_args *x, const pncxk_imap *m, int g)
{
    op *o;
    if (m->tmode != 0) return NODEV;              /* derived buftypes: not emulated */
    if ((o = new_op(do_imap)) == NULL) return NODEV;
    o->args = *x;
    o->i0 = k;
    o->i1 = a;
    o->i2 = b;
    o->i3 = g;
    o->n = (size_t)c;
    if ((o->b = malloc(sizeof *m)) == NULL) { free(o); return NODEV; }
    memcpy(o->b, m, sizeof *m);
    return enqueue(x->stream, o);
}
int pncxk_opinfo_get(int k, int a, int b, int c, pncxk_opinfo *o)
{
    (void)c;
    if (k == PNCXK_SWAP) {
        if (a != 1 && a != 2 && a != 4 && a != 8) return NODEV;
        o->ss = o->ds = a;
    } else if (k == PNCXK_GET) {
        o->ss = orc_xlen(a);
        o->ds = orc_ilen(b);
    } else if (k == PNCXK_PUT) {
        o->ss = orc_ilen(b);
        o->ds = orc_xlen(a);
    } else {
        return NODEV;
    }
    o->vec = 256;
    o->batch_steps = 1;
    return 0;
}
static void do_fill(op *o)
{
    long long i;
    check_access(o->a, o->n * (size_t)o->i0, "fill dst");
    for (i = 0; i < (long long)o->n; i++) memcpy((char *)o->a + i * o->i0, &o->args.fill, (size_t)o->i0);
}
int pncxk_fill(void *d, long long n, int x, const void *v, void *s)
{
    op *o = new_op(do_fill);
    if (o == NULL || x > 8) { free(o); return NODEV; }
    o->a = d;
    o->n = (size_t)n;
    o->i0 = x;
    memcpy(&o->args.fill, v, (size_t)x);
    return enqueue(s, o);
}
int pncxk_batch_map(const pncxk_batch_args *x) { (void)x; return 0; }
static void do_done(op *o)
{
    check_access(o->args.dst, sizeof(int), "completion word");
    if (o->i0 > 0) check_access(o->b, sizeof(int) * (size_t)o->i0, "status copy");
    if (o->i0 > 0) memcpy(o->b, o->a, sizeof(int) * (size_t)o->i0);
    __atomic_store_n((int *)o->args.dst, o->i1, __ATOMIC_RELEASE);
}
int pncxk_batch_done(const int *d, int n, int *h, int *w, int q, void *s)
{
    op *o = new_op(do_done);
    if (o == NULL) return NODEV;
    o->a = (void *)d;
    o->b = h;
    o->i0 = n;
    o->i1 = q;
    o->args.dst = w;
    return enqueue(s, o);
}
int pncxk_first_diff(const void *a, const void *b, long long n, int t, int tol, double td, double tr,
                     unsigned long long *f, void *s)
{ (void)a; (void)b; (void)n; (void)t; (void)tol; (void)td; (void)tr; (void)f; (void)s; return NODEV; }
