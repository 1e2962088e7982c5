/*
 * A synchronous CPU stand-in for the HIP shim (pncx_shim.h), used ONLY to
 * build the C host sources under ThreadSanitizer on a machine without a GPU
 * (tools/tsan/run.sh).  It is never linked into the library: its purpose is
 * to let the host code's device paths (staging area, pinned registration,
 * piece events, the nonblocking batch and its completion word, the warm-up
 * and enddef preload) run from many threads, so that the sanitizer sees every
 * access those paths make to shared host state.
 *
 * "Device" memory is malloc'ed and tracked so pointer queries answer as the
 * runtime would; copies run at once on the calling thread; streams and events
 * are tokens that are always complete.  Only byte swaps are carried out (the
 * same-type conversions the workload uses, and the batch kernels over them);
 * every other kernel reports no device, which the workload never reaches.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../../pnetcdf_amd/csrc/pncx_shim.h"

#define NODEV (-1900)

/* ---- device allocations (for pncxrt_is_device_ptr) ---- */
#define MAXALLOC 4096
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static struct { char *p; size_t n; } g_alloc[MAXALLOC];

static int find_alloc(const void *p)
{
    int i, r = -1;
    pthread_mutex_lock(&g_mu);
    for (i = 0; i < MAXALLOC && r < 0; i++)
        if (g_alloc[i].p && (const char *)p >= g_alloc[i].p && (const char *)p < g_alloc[i].p + g_alloc[i].n) r = i;
    pthread_mutex_unlock(&g_mu);
    return r;
}

int pncxrt_device_count(void) { return 1; }
int pncxrt_set_device(int dev) { return dev == 0 ? 0 : NODEV; }
int pncxrt_get_device(void) { return 0; }
int pncxrt_load_swap_code(void) { return 0; }
int pncxk_load_xtype(int x) { (void)x; return 0; }

int pncxrt_malloc(void **p, size_t n)
{
    int i;
    char *q = (char *)malloc(n ? n : 1);
    if (q == NULL) return NODEV;
    pthread_mutex_lock(&g_mu);
    for (i = 0; i < MAXALLOC && g_alloc[i].p; i++) {}
    if (i < MAXALLOC) { g_alloc[i].p = q; g_alloc[i].n = n ? n : 1; }
    pthread_mutex_unlock(&g_mu);
    if (i == MAXALLOC) { free(q); return NODEV; }
    *p = q;
    return 0;
}

int pncxrt_free(void *p)
{
    int i;
    if (p == NULL) return 0;
    pthread_mutex_lock(&g_mu);
    for (i = 0; i < MAXALLOC; i++)
        if (g_alloc[i].p == p) { g_alloc[i].p = NULL; g_alloc[i].n = 0; break; }
    pthread_mutex_unlock(&g_mu);
    free(p);
    return 0;
}

int pncxrt_host_alloc(void **p, size_t n) { return (*p = malloc(n ? n : 1)) ? 0 : NODEV; }
int pncxrt_host_alloc_mapped(void **p, void **dp, size_t n)
{
    *p = *dp = calloc(1, n ? n : 1);
    return *p ? 0 : NODEV;
}
int pncxrt_host_free(void *p) { free(p); return 0; }
int pncxrt_memcpy_h2d(void *d, const void *h, size_t n, void *s) { (void)s; memmove(d, h, n); return 0; }
int pncxrt_memcpy_d2h(void *h, const void *d, size_t n, void *s) { (void)s; memmove(h, d, n); return 0; }
int pncxrt_memcpy_d2d(void *d, const void *x, size_t n, void *s) { (void)s; memmove(d, x, n); return 0; }
int pncxrt_memset(void *d, int v, size_t n, void *s) { (void)s; memset(d, v, n); return 0; }

/* streams and events: tokens, always complete */
int pncxrt_stream_create(void **s) { return (*s = malloc(1)) ? 0 : NODEV; }
int pncxrt_stream_destroy(void *s) { free(s); return 0; }
int pncxrt_stream_sync(void *s) { (void)s; return 0; }
int pncxrt_event_create(void **e) { return (*e = malloc(1)) ? 0 : NODEV; }
int pncxrt_event_create_fast(void **e) { return pncxrt_event_create(e); }
int pncxrt_event_destroy(void *e) { free(e); return 0; }
int pncxrt_event_record(void *e, void *s) { (void)e; (void)s; return 0; }
int pncxrt_stream_wait_event(void *s, void *e) { (void)e; (void)s; return 0; }
int pncxrt_event_sync(void *e) { (void)e; return 0; }
int pncxrt_event_query(void *e) { (void)e; return 1; }
int pncxrt_event_elapsed_ms(float *ms, void *a, void *b) { (void)a; (void)b; *ms = 0.f; return 0; }

int pncxrt_is_device_ptr(const void *p) { return find_alloc(p) >= 0; }
int pncxrt_ptr_device(const void *p) { return find_alloc(p) >= 0 ? 0 : -1; }
/* registration: host memory is what the "device" reads, so every range maps to itself */
int pncxrt_host_register(void *p, size_t n) { (void)p; (void)n; return 0; }
int pncxrt_host_unregister(void *p) { (void)p; return 0; }
void *pncxrt_host_dptr(const void *p) { return (void *)p; }
void *pncxrt_host_dptr_range(const void *p, size_t n) { (void)n; return (void *)p; }
int pncxrt_host_register_map(void *p, size_t n, int r) { (void)p; (void)n; (void)r; return 0; }
const char *pncxrt_last_error(void) { return "CPU stand-in (ThreadSanitizer build)"; }

/* ---- kernels: byte swaps only ---- */
static long long g_nswap, g_nbatch, g_ndone;
/* launches so far (the workload prints them: the device paths did run) */
void cpudev_counts(long long *swap, long long *batch, long long *done)
{
    *swap = __atomic_load_n(&g_nswap, __ATOMIC_RELAXED);
    *batch = __atomic_load_n(&g_nbatch, __ATOMIC_RELAXED);
    *done = __atomic_load_n(&g_ndone, __ATOMIC_RELAXED);
}

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

int pncxk_swap(int e, const pncxk_args *a)
{
    if (e != 1 && e != 2 && e != 4 && e != 8) return NODEV;
    __atomic_add_fetch(&g_nswap, 1, __ATOMIC_RELAXED);
    swap_n(a->dst, a->src, a->n, e);
    return 0;
}
int pncxk_swap_generic(int e, const pncxk_args *a)
{
    if (e < 1 || e > 64) return NODEV;
    swap_n(a->dst, a->src, a->n, e);
    return 0;
}
int pncxk_get(int x, int i, const pncxk_args *a) { (void)x; (void)i; (void)a; return NODEV; }
int pncxk_put(int x, int i, int p, const pncxk_args *a) { (void)x; (void)i; (void)p; (void)a; return NODEV; }

int pncxk_batch(int k, int a, int b, int c, const pncxk_batch_args *x)
{
    int s;
    (void)b; (void)c;
    if (k != PNCXK_SWAP && k != PNCXK_SWAPMIX) return NODEV;
    __atomic_add_fetch(&g_nbatch, 1, __ATOMIC_RELAXED);
    for (s = 0; s < x->nseg; s++) {
        const pncxk_seg *g = &x->dsegs[s];
        swap_n(g->dst, g->src, g->n, k == PNCXK_SWAPMIX ? g->aux : a);
    }
    return 0;
}
int pncxk_batch_fused(int k, int a, int b, int c, const pncxk_batch_args *x, const pncxk_batch_args *y)
{ (void)k; (void)a; (void)b; (void)c; (void)x; (void)y; return NODEV; }
int pncxk_launch_imap(int k, int a, int b, int c, const pncxk_args *x, const pncxk_imap *m, int g)
{ (void)k; (void)a; (void)b; (void)c; (void)x; (void)m; (void)g; return NODEV; }
int pncxk_opinfo_get(int k, int a, int b, int c, pncxk_opinfo *o)
{
    (void)b; (void)c;
    if (k != PNCXK_SWAP || (a != 1 && a != 2 && a != 4 && a != 8)) return NODEV;
    o->ss = o->ds = a;
    o->vec = 4096 / a;
    o->batch_steps = 1;
    return 0;
}
int pncxk_fill(void *d, long long n, int x, const void *v, void *s)
{
    long long i;
    (void)s;
    for (i = 0; i < n; i++) memcpy((char *)d + i * x, v, (size_t)x);
    return 0;
}
int pncxk_batch_map(const pncxk_batch_args *x) { (void)x; return 0; }
int pncxk_batch_done(const int *d, int n, int *h, int *w, int q, void *s)
{
    (void)s;
    __atomic_add_fetch(&g_ndone, 1, __ATOMIC_RELAXED);
    if (n > 0) memcpy(h, d, sizeof(int) * (size_t)n);
    __atomic_store_n(w, q, __ATOMIC_RELEASE);
    return 0;
}
int pncxk_first_diff(const void *a, const void *b, long long n, int t, int tol, double td, double tr,
                     unsigned long long *f, void *s)
{ (void)a; (void)b; (void)n; (void)t; (void)tol; (void)td; (void)tr; (void)f; (void)s; return NODEV; }
