/*
 * Host-only stand-ins for the HIP shim (pncx_shim.h), used ONLY to build the
 * C host sources under AddressSanitizer on a machine without a GPU
 * (tools/asan/run.sh).  Every device operation reports no device, exactly
 * what the real shim returns when no GPU is visible, so the product code
 * takes its "no GPU" paths; nothing here converts data.
 */
#include <stdlib.h>
#include "../../pnetcdf_amd/csrc/pncx_shim.h"

#define NODEV (-1900)
int pncxrt_device_count(void) { return 0; }
int pncxrt_set_device(int dev) { (void)dev; return NODEV; }
int pncxrt_get_device(void) { return 0; }
int pncxrt_load_swap_code(void) { return NODEV; }
int pncxk_load_xtype(int x) { (void)x; return NODEV; }
int pncxrt_malloc(void **p, size_t n) { (void)p; (void)n; return NODEV; }
int pncxrt_free(void *p) { (void)p; return 0; }
int pncxrt_host_alloc(void **p, size_t n) { (void)p; (void)n; return NODEV; }
int pncxrt_host_alloc_mapped(void **p, void **dp, size_t n) { (void)p; (void)dp; (void)n; return NODEV; }
int pncxrt_host_free(void *p) { (void)p; return 0; }
int pncxrt_memcpy_h2d(void *d, const void *h, size_t n, void *s) { (void)d; (void)h; (void)n; (void)s; return NODEV; }
int pncxrt_memcpy_d2h(void *h, const void *d, size_t n, void *s) { (void)d; (void)h; (void)n; (void)s; return NODEV; }
int pncxrt_memcpy_d2d(void *d, const void *x, size_t n, void *s) { (void)d; (void)x; (void)n; (void)s; return NODEV; }
int pncxrt_memset(void *d, int v, size_t n, void *s) { (void)d; (void)v; (void)n; (void)s; return NODEV; }
int pncxrt_stream_create(void **s) { (void)s; return NODEV; }
int pncxrt_stream_destroy(void *s) { (void)s; return 0; }
int pncxrt_stream_sync(void *s) { (void)s; return NODEV; }
int pncxrt_event_create(void **e) { (void)e; return NODEV; }
int pncxrt_event_create_fast(void **e) { (void)e; return NODEV; }
int pncxrt_event_destroy(void *e) { (void)e; return 0; }
int pncxrt_event_record(void *e, void *s) { (void)e; (void)s; return NODEV; }
int pncxrt_stream_wait_event(void *s, void *e) { (void)e; (void)s; return NODEV; }
int pncxrt_event_sync(void *e) { (void)e; return NODEV; }
int pncxrt_event_query(void *e) { (void)e; return NODEV; }
int pncxrt_event_elapsed_ms(float *ms, void *a, void *b) { (void)ms; (void)a; (void)b; return NODEV; }
int pncxrt_is_device_ptr(const void *p) { (void)p; return 0; }
int pncxrt_ptr_device(const void *p) { (void)p; return -1; }
int pncxrt_host_register(void *p, size_t n) { (void)p; (void)n; return NODEV; }
int pncxrt_host_unregister(void *p) { (void)p; return 0; }
void *pncxrt_host_dptr(const void *p) { (void)p; return NULL; }
void *pncxrt_host_dptr_range(const void *p, size_t n) { (void)p; (void)n; return NULL; }
int pncxrt_host_register_map(void *p, size_t n, int r) { (void)p; (void)n; (void)r; return NODEV; }
const char *pncxrt_last_error(void) { return "no device (host-only ASan build)"; }
int pncxk_swap(int e, const pncxk_args *a) { (void)e; (void)a; return NODEV; }
int pncxk_swap_generic(int e, const pncxk_args *a) { (void)e; (void)a; return NODEV; }
int pncxk_get(int x, int i, const pncxk_args *a) { (void)x; (void)i; (void)a; return NODEV; }
int pncxk_put(int x, int i, int p, const pncxk_args *a) { (void)x; (void)i; (void)p; (void)a; return NODEV; }
int pncxk_batch(int k, int a, int b, int c, const pncxk_batch_args *x) { (void)k; (void)a; (void)b; (void)c; (void)x; return NODEV; }
int pncxk_batch_fused(int k, int a, int b, int c, const pncxk_batch_args *x, const pncxk_batch_args *y)
{ (void)k; (void)a; (void)b; (void)c; (void)x; (void)y; return NODEV; }
int pncxk_launch_imap(int k, int a, int b, int c, const pncxk_args *x, const pncxk_imap *m, int g)
{ (void)k; (void)a; (void)b; (void)c; (void)x; (void)m; (void)g; return NODEV; }
int pncxk_opinfo_get(int k, int a, int b, int c, pncxk_opinfo *o) { (void)k; (void)a; (void)b; (void)c; (void)o; return NODEV; }
int pncxk_fill(void *d, long long n, int x, const void *v, void *s) { (void)d; (void)n; (void)x; (void)v; (void)s; return NODEV; }
int pncxk_batch_map(const pncxk_batch_args *x) { (void)x; return NODEV; }
int pncxk_batch_done(const int *d, int n, int *h, int *w, int q, void *s) { (void)d; (void)n; (void)h; (void)w; (void)q; (void)s; return NODEV; }
int pncxk_first_diff(const void *a, const void *b, long long n, int t, int tol, double td, double tr,
                     unsigned long long *f, void *s)
{ (void)a; (void)b; (void)n; (void)t; (void)tol; (void)td; (void)tr; (void)f; (void)s; return NODEV; }
