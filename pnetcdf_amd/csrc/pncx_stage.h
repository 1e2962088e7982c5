/*
 * pncx_stage.h -- chunked, asynchronous conversion of host buffers through
 * HBM (internal to libpncx.so: pncx_host.c implements it, the host-buffer
 * entry points and the file layer's put/get pipelines in pncx_nc.c use it).
 *
 *   pncx_stage_begin(&h, PNCX_PUT, cdf, xtype, itype, fill, chunk_elems, total_elems);
 *   k = pncx_stage_push(h, src, dst, n);   enqueue H2D, kernel, D2H of one chunk
 *   pncx_stage_wait(h, k);                  chunk k's bytes are in dst
 *   st = pncx_stage_end(h);                 wait all; first status (NC_ERANGE)
 *
 * The reference converts a request in one pass on the calling thread
 * (ncmpio_pack_xbuf / ncmpio_unpack_xbuf, ncmpio_util.c:716-765,842-888);
 * here the file I/O of chunk k runs while chunk k+1 is still converting.
 * The handle holds the device's staging context from begin to end: other
 * host-buffer conversions of the process wait for it.  Host memory should
 * be pinned (hipHostMalloc) or registered; pageable memory works but its
 * copies are not asynchronous.
 */
#ifndef PNCX_STAGE_H
#define PNCX_STAGE_H

#ifdef __cplusplus
extern "C" {
#endif

#define PNCX_SWAP_DIR 3    /* dir of a plain swap: xtype = element size, itype unused */

typedef struct pncx_stage pncx_stage;
int pncx_stage_begin(pncx_stage **h, int dir, int cdf_ver, int xtype, int itype, const void *fillp,
                     long long max_chunk_elems, long long total_elems);
int pncx_stage_push(pncx_stage *h, const void *src, void *dst, long long nelems);
int pncx_stage_wait(pncx_stage *h, int k);
int pncx_stage_end(pncx_stage *h);
long long pncx_stage_chunk(const pncx_stage *h);
/* [p, p + n) is one device-accessible host range for the rest of the call
 * (the registered user buffer, the pinned staging area): pushes inside it
 * skip the runtime's pointer lookups */
void pncx_stage_hint(pncx_stage *h, const void *p, size_t n);

/* one conversion launch between device-accessible pointers (HBM, pinned or
 * registered host memory, a registered file window), waited for: the
 * status (NC_ERANGE) or an error.  after: NULL, or the address of a stream
 * handle (the caller's; a NULL handle is the legacy default stream) whose
 * queued work the launch must follow */
int pncx_direct_convert(int dir, int cdf_ver, int xtype, int itype, const void *fillp, const void *dsrc,
                        void *ddst, long long nelems, void *const *after);

#ifdef __cplusplus
}
#endif
#endif
