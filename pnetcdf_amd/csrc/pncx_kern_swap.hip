// pncx_kern_swap.hip -- byte-swap / copy launchers, the generic n-byte swap
// kernel, grid sizing, batch dispatch, and the thin HIP-runtime wrappers that
// the C host code (pncx_host.c) calls.
#include <stdlib.h>
#include <string.h>

#include <pthread.h>

#include <mutex>

#include "pncx_kern.hpp"

using namespace pncx;

// ---------------------------------------------------------------------------
// grid sizing: memory-bound streaming -> enough blocks to fill 256 CUs
// (8 XCDs x 32 CUs) several times, grid-stride the rest.
// ---------------------------------------------------------------------------
static int g_cu_count[64];

static int cu_count() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    // set by whichever thread asks first; every thread computes the same value
    int cus = __atomic_load_n(&g_cu_count[dev], __ATOMIC_RELAXED);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        __atomic_store_n(&g_cu_count[dev], cus, __ATOMIC_RELAXED);
    }
    return cus;
}

static int blocks_per_cu() {
    static int v = -1;
    int b = __atomic_load_n(&v, __ATOMIC_RELAXED);
    if (b < 0) {
        const char *e = getenv("PNCX_BLOCKS_PER_CU");
        b = (e && atoi(e) > 0) ? atoi(e) : 8;
        __atomic_store_n(&v, b, __ATOMIC_RELAXED);
    }
    return b;
}

namespace pncx {
int launch_grid(int64_t work_items, int per_thread) {
    const int64_t want = (work_items + 256LL * per_thread - 1) / (256LL * per_thread);
    const int64_t cap = (int64_t)cu_count() * blocks_per_cu();
    int64_t g = want < cap ? want : cap;
    if (g < 1) g = 1;
    return (int)g;
}
}  // namespace pncx

// ---------------------------------------------------------------------------
// generic esize (not 1/2/4/8): one element per lane, byte reversal
// (ncmpii_in_swapn generic branch, convert_swap.m4:184-195)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_swap_generic(const uint8_t *src, uint8_t *dst, int64_t n,
                                                      int esize) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = tid; e < n; e += stride) {
        const uint8_t *s = src + e * esize;
        uint8_t *d = dst + e * esize;
        for (int i = 0; i < esize / 2; i++) {
            const uint8_t a = s[i], b = s[esize - 1 - i];
            d[i] = b;
            d[esize - 1 - i] = a;
        }
        if (esize & 1) d[esize / 2] = s[esize / 2];
    }
}

extern "C" int pncxk_swap(int esize, const pncxk_args *a) {
    switch (esize) {
        case 1: return launch_stream<SwapOp<1>>(a);
        case 2: return launch_stream<SwapOp<2>>(a);
        case 4: return launch_stream<SwapOp<4>>(a);
        case 8: return launch_stream<SwapOp<8>>(a);
        default: return pncxk_swap_generic(esize, a);
    }
}

extern "C" int pncxk_swap_generic(int esize, const pncxk_args *a) {
    if (a->n <= 0 || esize <= 0) return 0;
    const int grid = launch_grid(a->n, 1);
    hipLaunchKernelGGL(k_swap_generic, dim3(grid), dim3(256), 0, (hipStream_t)a->stream,
                       (const uint8_t *)a->src, (uint8_t *)a->dst, (int64_t)a->n, esize);
    return hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE;
}

// ---------------------------------------------------------------------------
// fill_var_buf (ncmpio_fill.c:89-140): replicate one xsize-byte external
// (big-endian) fill value over the buffer.  Pure write: one-shot grid, one
// nontemporal 16 B store per lane (16 is a multiple of every xsize), scalar
// bytes before the first 128 B boundary and after the last 16 B vector.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fill(uint8_t *dst, int64_t nbytes, int64_t head, int64_t nvec,
                                              u32x4 pattern, uint64_t xvalue, int xsize) {
    const int64_t nb = gridDim.x;
    if (blockIdx.x == 0) {
        const int64_t tail0 = head + nvec * 16;
        for (int64_t j = threadIdx.x; j < head; j += 256) dst[j] = (uint8_t)(xvalue >> (8 * (j % xsize)));
        for (int64_t j = tail0 + threadIdx.x; j < nbytes; j += 256)
            dst[j] = (uint8_t)(xvalue >> (8 * (j % xsize)));
    }
    u32x4 *v = reinterpret_cast<u32x4 *>(dst + head);
    for (int64_t k = xcd_remap(blockIdx.x, nb) * 256 + threadIdx.x; k < nvec; k += nb * 256)
        st_stream<u32x4>(reinterpret_cast<uint8_t *>(v + k), pattern);
}

extern "C" int pncxk_fill(void *dst, long long nelems, int xsize, const void *xvalue, void *stream) {
    if (nelems <= 0) return 0;
    if (xsize != 1 && xsize != 2 && xsize != 4 && xsize != 8) return NC_EINVAL;
    uint64_t xv = 0;
    memcpy(&xv, xvalue, (size_t)xsize);                  // external bytes, in memory order
    const int64_t nbytes = (int64_t)nelems * xsize;
    const uintptr_t a = (uintptr_t)dst;
    // the vector body starts on a 128-byte line: with a 16-byte-aligned but
    // line-misaligned start every wave store splits 9 lines and the rate
    // drops from 6.96 to 5.49 TB/s (tools/fill_bench.py, 3-byte offset)
    int64_t head = (int64_t)((128 - (a & 127)) & 127);
    if (head > nbytes) head = nbytes;
    const int64_t nvec = (nbytes - head) / 16;
    uint8_t pb[16];
    for (int b = 0; b < 16; b++) pb[b] = (uint8_t)(xv >> (8 * ((head + b) % xsize)));
    u32x4 pattern;
    memcpy(&pattern, pb, 16);
    int64_t grid = (nvec + 255) / 256;
    if (grid < 1) grid = 1;
    if (grid > MAX_BLOCKS) grid = MAX_BLOCKS;
    hipLaunchKernelGGL(k_fill, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, (uint8_t *)dst, nbytes,
                       head, nvec, pattern, xv, xsize);
    return hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE;
}

// ---------------------------------------------------------------------------
// NC_ERANGE reporting through per-block flags (see Sink in pncx_kern.hpp).
// A flag array belongs to one (device, stream[, thread]): calls on one stream
// run in order, so each call's epoch is new to its array and no zeroing is
// needed; calls on different streams never share an array (sharing one would
// let a later call overwrite an earlier call's flags before its reduce reads
// them).  hipStreamPerThread is one handle for many streams (one per host
// thread), so its slots are also keyed by the calling thread.
// The mutex is held from sink_acquire to sink_finish so that one call's
// kernel and reduce are enqueued back to back; nothing waits on the device
// while it is held.
// No event marks a reduce's completion: an event recorded after every reduce
// delayed the next kernel on the stream by 5.8 us (the synchronous batch's
// completion kernel, profiles/r02s_c4_erange trace).  So an array can only be
// known unread once its device has drained: a slot taken over by another
// stream (more than NFLAGSLOT streams in use) or regrown gets a fresh zeroed
// array, and the old one is retired and freed after the mutex is released
// (hipFree drains the device itself).
// ---------------------------------------------------------------------------
namespace {
struct FlagSlot {
    int dev;
    hipStream_t stream;
    pthread_t thread;     // the owning thread, for hipStreamPerThread only
    int *flags;
    int64_t cap;          // ints
    int epoch;
    uint64_t tick;
    bool live;
};
struct Retired {
    int dev;
    int *flags;
};
constexpr int NFLAGSLOT = 32;
constexpr int NRETIRE = 2 * NFLAGSLOT;
FlagSlot g_fslot[NFLAGSLOT];
Retired g_retired[NRETIRE];
int g_nretired;
std::mutex g_fslot_mu;
uint64_t g_ftick;

bool same_owner(const FlagSlot *c, int dev, hipStream_t st, pthread_t self) {
    return c->live && c->dev == dev && c->stream == st && (st != hipStreamPerThread || pthread_equal(c->thread, self));
}

// queue an array for freeing once the mutex is dropped (caller holds it).
// Every release frees the list, and one acquire retires at most two arrays,
// so the list cannot fill up; if it ever did, the array is freed here, under
// the mutex (hipFree drains the device first, so no queued kernel or reduce
// still reads it) rather than leaked.
void retire(int dev, int *flags) {
    if (flags == nullptr) return;
    if (g_nretired >= NRETIRE) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (dev != cur) (void)hipSetDevice(dev);
        (void)hipFree(flags);
        if (dev != cur) (void)hipSetDevice(cur);
        return;
    }
    g_retired[g_nretired++] = Retired{dev, flags};
}

// free retired arrays with the mutex released: hipFree waits for the device
// (the kernels and reduces that read them) without blocking other launches
void free_retired() {
    Retired r[NRETIRE];
    int n;
    {
        std::lock_guard<std::mutex> g(g_fslot_mu);
        n = g_nretired;
        for (int i = 0; i < n; i++) r[i] = g_retired[i];
        g_nretired = 0;
    }
    if (n == 0) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (int i = 0; i < n; i++) {
        if (r[i].dev != cur) (void)hipSetDevice(r[i].dev);
        (void)hipFree(r[i].flags);
        if (r[i].dev != cur) (void)hipSetDevice(cur);
    }
}
}  // namespace

namespace pncx {

Sink sink_acquire(int *status, int sval, hipStream_t st, int64_t nblocks, bool want) {
    Sink s{status, nullptr, 0, sval};
    if (!want || nblocks <= 0) return s;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return s;
    const pthread_t self = pthread_self();
    g_fslot_mu.lock();
    FlagSlot *f = nullptr, *lru = nullptr;
    for (int i = 0; i < NFLAGSLOT; i++) {
        FlagSlot *c = &g_fslot[i];
        if (same_owner(c, dev, st, self)) { f = c; break; }
        if (lru == nullptr || !c->live || (lru->live && c->tick < lru->tick)) lru = c;
    }
    if (f == nullptr) {                 // take a free slot, or the least recently used one
        f = lru;
        if (f->live) {                  // its last reduce may still be queued: retire the array
            retire(f->dev, f->flags);
            f->flags = nullptr;
            f->cap = 0;
        }
        f->live = true;
        f->dev = dev;
        f->stream = st;
        f->thread = self;
    }
    if (f->cap < nblocks) {             // grow: the old array may still be read on this stream
        retire(f->dev, f->flags);
        f->flags = nullptr;
        f->cap = nblocks > 2 * f->cap ? nblocks : 2 * f->cap;
    }
    if (f->flags == nullptr) {
        if (hipMalloc(&f->flags, sizeof(int) * (size_t)f->cap) != hipSuccess ||
            hipMemsetAsync(f->flags, 0, sizeof(int) * (size_t)f->cap, st) != hipSuccess) {
            (void)hipGetLastError();
            if (f->flags) retire(dev, f->flags);
            f->flags = nullptr;
            f->cap = 0;
            f->live = false;
            g_fslot_mu.unlock();
            free_retired();
            return s;                   // per-wave publish
        }
        f->epoch = 0;                   // a zeroed array: any epoch >= 1 is new to it
    }
    if (++f->epoch >= 0x3fffffff) {     // epochs must not repeat on this array
        if (hipMemsetAsync(f->flags, 0, sizeof(int) * (size_t)f->cap, st) != hipSuccess) {
            g_fslot_mu.unlock();
            free_retired();
            return s;
        }
        f->epoch = 1;
    }
    f->tick = ++g_ftick;
    s.flags = f->flags;
    s.epoch = f->epoch;
    return s;                           // the mutex stays held until sink_finish*
}

static void sink_release(hipStream_t) {
    const bool pending = g_nretired > 0;
    g_fslot_mu.unlock();
    if (pending) free_retired();
}

}  // namespace pncx

namespace pncx {
// A/B knobs: read once at load, pncx_knob_set in tests (pncx_shim.h)
int tile_u(int dflt) {
    const long long v = pncx_knob(PNCXK_KNOB_TILE_U);
    return v == 1 || v == 2 || v == 4 ? (int)v : dflt;
}
int xpose_merge() { return pncx_knob(PNCXK_KNOB_XPOSE_MERGE) != 0; }
int xpose_order() { const long long v = pncx_knob(PNCXK_KNOB_XPOSE_ORDER); return v < 0 ? -1 : (int)v; }
int urun_enabled() { return pncx_knob(PNCXK_KNOB_URUN) != 0; }
int tmap_vec() { return pncx_knob(PNCXK_KNOB_TMAP_VEC) != 0; }
int imap_rows() { return pncx_knob(PNCXK_KNOB_IMAP_ROWS) != 0; }
int tgap_enabled() { return pncx_knob(PNCXK_KNOB_TGAP) != 0; }
int fuse_lanes() { return pncx_knob(PNCXK_KNOB_FUSE_LANES) == 1024 ? 1024 : 256; }
}  // namespace pncx

// single status word: any flag of this launch's epoch -> *status = sval
__global__ __launch_bounds__(256) void k_flags_one(const int *flags, int64_t nb, int epoch, int *status, int sval) {
    bool hit = false;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += (int64_t)gridDim.x * 256)
        hit |= flags[i] == epoch;
    if (__syncthreads_or(hit) && threadIdx.x == 0 &&
        __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != sval)
        __hip_atomic_store(status, sval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// batch: one block per segment over its blocks [block0, next block0)
__global__ __launch_bounds__(256) void k_flags_batch(const pncxk_seg *segs, int nseg, int64_t nb, const int *flags,
                                                     int epoch, int sval) {
    const int s = blockIdx.x;
    if (s >= nseg) return;                 // whole block leaves together
    const int64_t b0 = segs[s].block0, b1 = s + 1 < nseg ? segs[s + 1].block0 : nb;
    bool hit = false;
    for (int64_t b = b0 + threadIdx.x; b < b1; b += 256) hit |= flags[b] == epoch;
    int *st = segs[s].status;
    if (__syncthreads_or(hit) && threadIdx.x == 0 && st != nullptr) *st = sval;
}

namespace pncx {

int sink_finish(const Sink &s, hipStream_t st, int64_t nblocks, int err) {
    if (s.flags == nullptr) return err;
    if (!err) {
        int64_t g = (nblocks + 255) / 256;       /* one flag per lane up to 2^18 blocks */
        if (g > 1024) g = 1024;
        if (g < 1) g = 1;
        hipLaunchKernelGGL(k_flags_one, dim3((unsigned)g), dim3(256), 0, st, s.flags, nblocks, s.epoch, s.status,
                           s.sval);
        if (hipGetLastError() != hipSuccess) err = PNCX_EDEVICE;
    }
    sink_release(st);
    return err;
}

int sink_finish_batch(const Sink &s, const pncxk_seg *dsegs, int nseg, int64_t nblocks, hipStream_t st, int err) {
    if (s.flags == nullptr) return err;
    if (!err && nseg > 0) {
        hipLaunchKernelGGL(k_flags_batch, dim3((unsigned)nseg), dim3(256), 0, st, dsegs, nseg, nblocks, s.flags,
                           s.epoch, s.sval);
        if (hipGetLastError() != hipSuccess) err = PNCX_EDEVICE;
    }
    sink_release(st);
    return err;
}

}  // namespace pncx

// batch / opinfo dispatch: get and put live in their own TUs
extern "C" int pncxk_batch_get(int xtype, int itype, const pncxk_batch_args *a);
extern "C" int pncxk_batch_put(int xtype, int itype, int preserve, const pncxk_batch_args *a);
extern "C" int pncxk_opinfo_getput(int kind, int xtype, int itype, int preserve, pncxk_opinfo *o);

// One launch for all same-type segments of a batch (C4: NC_SHORT and
// NC_FLOAT iputs): the block's segment says its element size (mix_block,
// pncx_kern.hpp).  A block is MIX_LANES lanes x 16 B (one nontemporal vector
// each, no loop), blocks in XCD-contiguous order.  Round 2
// (tools/c4_shape_sweep.hip, 256 buffer pairs, splitmix64 data, three
// boxes): launch order at 1024 lanes 75.8-77.1 % of peak, XCD-contiguous
// order 80.3-82.7 % at 256, 512 or 1024 lanes; the same descriptors pointing
// into one allocation per side 83.3-84.1 %, one flat buffer pair 83.4-84.5 %.
// Two or four vectors per lane lose 1-5 points.  Plain (write-back) stores
// lose 1-4 points to "nt sc1" in the library (tools/c4_placement.py);
// persistent grids that prefetch their next tile ran at 65-74 %
// (tools/c4_store_sweep.hip).
__global__ __launch_bounds__(MIX_LANES) void k_batch_swapmix(const pncxk_seg *segs, int nseg, const int *map,
                                                             pncxk_groups grp) {
    mix_block(segs, nseg, map, grp, batch_block());
}

extern "C" int pncxk_batch(int kind, int a, int b, int c, const pncxk_batch_args *args) {
    if (kind == PNCXK_SWAPMIX) {
        if (args->nblocks <= 0) return 0;
        auto k = k_batch_swapmix;
        if (args->ev_start != nullptr || args->ev_stop != nullptr)
            hipExtLaunchKernelGGL(k, dim3((unsigned)args->nblocks), dim3(MIX_LANES), 0,
                                  (hipStream_t)args->stream, (hipEvent_t)args->ev_start, (hipEvent_t)args->ev_stop, 0,
                                  args->dsegs, args->nseg, args->dmap, args->grp);
        else
            hipLaunchKernelGGL(k, dim3((unsigned)args->nblocks), dim3(MIX_LANES), 0,
                               (hipStream_t)args->stream, args->dsegs, args->nseg, args->dmap, args->grp);
        return hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE;
    }
    if (kind == PNCXK_SWAP) {
        switch (a) {
            case 1: return launch_batch<SwapOp<1>>(args);
            case 2: return launch_batch<SwapOp<2>>(args);
            case 4: return launch_batch<SwapOp<4>>(args);
            case 8: return launch_batch<SwapOp<8>>(args);
            default: return NC_EINVAL;
        }
    }
    if (kind == PNCXK_GET) return pncxk_batch_get(a, b, args);
    if (kind == PNCXK_PUT) return pncxk_batch_put(a, b, c, args);
    return NC_EINVAL;
}

extern "C" int pncxk_batch_fused_get(int xtype, int itype, const pncxk_batch_args *a, const pncxk_batch_args *m);
extern "C" int pncxk_batch_fused_put(int xtype, int itype, int preserve, const pncxk_batch_args *a,
                                     const pncxk_batch_args *m);

extern "C" int pncxk_batch_fused(int kind, int a, int b, int c, const pncxk_batch_args *conv,
                                 const pncxk_batch_args *mix) {
    if (kind == PNCXK_GET) return pncxk_batch_fused_get(a, b, conv, mix);
    if (kind == PNCXK_PUT) return pncxk_batch_fused_put(a, b, c, conv, mix);
    return PNCXK_NOFUSE;
}

// block -> segment table for non-uniform batches: block s of this grid
// writes s into [seg[s].block0, seg[s].block0 + nblocks(s))
static __global__ __launch_bounds__(256) void k_batch_map(const pncxk_seg *segs, int nseg, long long nblocks,
                                                   int *map) {
    const int s = blockIdx.x;
    if (s >= nseg) return;
    const long long b0 = segs[s].block0;
    const long long b1 = s + 1 < nseg ? segs[s + 1].block0 : nblocks;
    for (long long b = b0 + threadIdx.x; b < b1; b += 256) map[b] = s;
}

extern "C" int pncxk_imap_get(int xtype, int itype, const pncxk_args *a, const pncxk_imap *m);
extern "C" int pncxk_imap_put(int xtype, int itype, int preserve, const pncxk_args *a, const pncxk_imap *m);

extern "C" int pncxk_launch_imap(int kind, int a, int b, int c, const pncxk_args *args, const pncxk_imap *m,
                          int gather) {
    if (kind == PNCXK_SWAP) {
        switch (a) {
            case 1: return launch_imap<SwapOp<1>>(args, m, gather);
            case 2: return launch_imap<SwapOp<2>>(args, m, gather);
            case 4: return launch_imap<SwapOp<4>>(args, m, gather);
            case 8: return launch_imap<SwapOp<8>>(args, m, gather);
            default: return NC_EINVAL;
        }
    }
    if (kind == PNCXK_GET) return pncxk_imap_get(a, b, args, m);
    if (kind == PNCXK_PUT) return pncxk_imap_put(a, b, c, args, m);
    return NC_EINVAL;
}

extern "C" int pncxk_batch_map(const pncxk_batch_args *a) {
    if (a->nseg <= 0 || a->dmap == nullptr) return 0;
    hipLaunchKernelGGL(k_batch_map, dim3((unsigned)a->nseg), dim3(256), 0, (hipStream_t)a->stream,
                       a->dsegs, a->nseg, a->nblocks, a->dmap);
    return hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE;
}

// Completion of a synchronous pncx_dev_batch: the statuses go straight into
// host-mapped (fine-grained) memory and a sequence word follows them, which
// the host polls -- no status copy command and no completion event.  A
// 768 MiB swap kernel waited for this way took 257 us per call against 260
// with hipEventRecord + hipEventQuery and 248 back to back
// (tools/turnaround_probe.hip, profiles/r02_turnaround_probe.txt).  One
// block; vector stores only.
__global__ __launch_bounds__(256) void k_batch_done(const int *dstat, int n, int *hstat, int *hdone, int seq) {
    for (int i = threadIdx.x; i < n; i += 256) __hip_atomic_store(hstat + i, dstat[i], __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(hdone, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A batch with no statuses to bring back (swaps and copies only) has
// nothing for a system-scope release to order before the flag -- the class
// kernels' stores were released at their own end, before this kernel
// started -- so one wave stores the flag relaxed: 0.7-0.8 us less per
// synchronous call (C4 0.2570 -> 0.2562 ms through bench.py's loop, a
// trivial call 10.0-11.5 -> 9.4-10.9 us from C; profiles/r06l_done_fence_ab.txt)
__global__ __launch_bounds__(64) void k_batch_done_flag(int *hdone, int seq) {
    if (threadIdx.x == 0) __hip_atomic_store(hdone, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" int pncxk_batch_done(const int *dstat, int n, int *hstat, int *hdone, int seq, void *stream) {
    if (n == 0)
        hipLaunchKernelGGL(k_batch_done_flag, dim3(1), dim3(64), 0, (hipStream_t)stream, hdone, seq);
    else
        hipLaunchKernelGGL(k_batch_done, dim3(1), dim3(256), 0, (hipStream_t)stream, dstat, n, hstat, hdone, seq);
    return hipGetLastError() == hipSuccess ? 0 : PNCX_EDEVICE;
}

extern "C" int pncxk_opinfo_get(int kind, int a, int b, int c, pncxk_opinfo *o) {
    if (kind == PNCXK_SWAP) {
        switch (a) {
            case 1: OpInfo<SwapOp<1>>::fill(o); return 0;
            case 2: OpInfo<SwapOp<2>>::fill(o); return 0;
            case 4: OpInfo<SwapOp<4>>::fill(o); return 0;
            case 8: OpInfo<SwapOp<8>>::fill(o); return 0;
            default: return NC_EINVAL;
        }
    }
    return pncxk_opinfo_getput(kind, a, b, c, o);
}

// ---------------------------------------------------------------------------
// HIP runtime wrappers
// ---------------------------------------------------------------------------
static thread_local char g_last_err[256];

static int rt(hipError_t e, const char *what) {
    if (e == hipSuccess) return 0;
    snprintf(g_last_err, sizeof g_last_err, "%s: %s", what, hipGetErrorString(e));
    return PNCX_EDEVICE;
}

extern "C" {
const char *pncxrt_last_error(void) { return g_last_err; }
int pncxrt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
int pncxrt_set_device(int dev) { return rt(hipSetDevice(dev), "hipSetDevice"); }
// HIP loads a code object on a device at the first launch from it; a
// function-attribute query loads it too.  This file's (the same-type swaps
// and copies, the batch and fill kernels: 1.2 MB) costs 4-5 ms, which the
// create/open warm-up (pncx_warmup) takes off a process's first put; the
// per-type conversion objects stay lazy (~18 ms each, pncx_kern_xt.c)
int pncxrt_load_swap_code(void) {
    hipFuncAttributes fa;
    return rt(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&k_swap_generic)), "hipFuncGetAttributes");
}
int pncxrt_get_device(void) {
    int d = -1;
    if (hipGetDevice(&d) != hipSuccess) return -1;
    return d;
}
int pncxrt_malloc(void **p, size_t n) { return rt(hipMalloc(p, n ? n : 1), "hipMalloc"); }
int pncxrt_free(void *p) { return p ? rt(hipFree(p), "hipFree") : 0; }
int pncxrt_host_alloc(void **p, size_t n) {
    return rt(hipHostMalloc(p, n ? n : 1, hipHostMallocDefault), "hipHostMalloc");
}
int pncxrt_host_alloc_mapped(void **p, void **dp, size_t n) {
    *p = *dp = nullptr;
    if (rt(hipHostMalloc(p, n ? n : 1, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc coherent"))
        return PNCX_EDEVICE;
    if (rt(hipHostGetDevicePointer(dp, *p, 0), "hipHostGetDevicePointer")) {
        (void)hipHostFree(*p);
        *p = *dp = nullptr;
        return PNCX_EDEVICE;
    }
    return 0;
}
int pncxrt_host_free(void *p) { return p ? rt(hipHostFree(p), "hipHostFree") : 0; }
int pncxrt_memcpy_h2d(void *d, const void *h, size_t n, void *s) {
    return rt(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, (hipStream_t)s), "hipMemcpyAsync H2D");
}
int pncxrt_memcpy_d2h(void *h, const void *d, size_t n, void *s) {
    return rt(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, (hipStream_t)s), "hipMemcpyAsync D2H");
}
int pncxrt_memcpy_d2d(void *d, const void *src, size_t n, void *s) {
    return rt(hipMemcpyAsync(d, src, n, hipMemcpyDeviceToDevice, (hipStream_t)s), "hipMemcpyAsync D2D");
}
int pncxrt_memset(void *d, int v, size_t n, void *s) {
    return rt(hipMemsetAsync(d, v, n, (hipStream_t)s), "hipMemsetAsync");
}
int pncxrt_stream_create(void **s) {
    return rt(hipStreamCreateWithFlags((hipStream_t *)s, hipStreamNonBlocking), "hipStreamCreate");
}
int pncxrt_stream_destroy(void *s) { return s ? rt(hipStreamDestroy((hipStream_t)s), "hipStreamDestroy") : 0; }
int pncxrt_stream_sync(void *s) { return rt(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize"); }
int pncxrt_event_create(void **e) { return rt(hipEventCreate((hipEvent_t *)e), "hipEventCreate"); }
int pncxrt_event_create_fast(void **e) {
    return rt(hipEventCreateWithFlags((hipEvent_t *)e, hipEventDisableTiming), "hipEventCreateWithFlags");
}
int pncxrt_event_destroy(void *e) { return e ? rt(hipEventDestroy((hipEvent_t)e), "hipEventDestroy") : 0; }
int pncxrt_event_record(void *e, void *s) {
    return rt(hipEventRecord((hipEvent_t)e, (hipStream_t)s), "hipEventRecord");
}
int pncxrt_stream_wait_event(void *s, void *e) {
    return rt(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)e, 0), "hipStreamWaitEvent");
}
int pncxrt_event_sync(void *e) { return rt(hipEventSynchronize((hipEvent_t)e), "hipEventSynchronize"); }
int pncxrt_event_elapsed_ms(float *ms, void *a, void *b) {
    return rt(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b), "hipEventElapsedTime");
}
int pncxrt_event_query(void *e) {
    const hipError_t r = hipEventQuery((hipEvent_t)e);
    if (r == hipSuccess) return 1;
    if (r == hipErrorNotReady) { (void)hipGetLastError(); return 0; }
    return rt(r, "hipEventQuery");
}
int pncxrt_host_register(void *p, size_t n) {
    /* hipHostRegister on an already registered range returns success and a
     * later unregister would drop the owner's registration: look first */
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) == hipSuccess &&
        (at.type == hipMemoryTypeHost || at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged))
        return 1;
    (void)hipGetLastError();
    if (hipHostRegister(p, n, hipHostRegisterMapped) == hipSuccess) return 0;
    (void)hipGetLastError();
    return PNCX_EDEVICE;
}
int pncxrt_host_unregister(void *p) { return rt(hipHostUnregister(p), "hipHostUnregister"); }
int pncxrt_host_register_map(void *p, size_t n, int readonly) {
    unsigned fl = hipHostRegisterMapped | (readonly ? hipHostRegisterReadOnly : 0u);
    if (hipHostRegister(p, n, fl) == hipSuccess) return 0;
    (void)hipGetLastError();
    if (readonly && hipHostRegister(p, n, hipHostRegisterMapped) == hipSuccess) return 0;
    (void)hipGetLastError();
    return PNCX_EDEVICE;
}
void *pncxrt_host_dptr_range(const void *p, size_t n) {
    /* the device address of [p, p + n) when the whole range lies inside ONE
     * pinned or registered host allocation, else NULL: a range that starts
     * inside one registration and runs past its end, or spans two
     * registrations with pageable memory between them, must not reach a
     * kernel.  The runtime's range of the allocation holding p
     * (HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR / _SIZE: the registration
     * itself for hipHostRegister'ed memory, tools/ptr_range_probe.hip,
     * profiles/r05b_ptr_range_probe.txt) must contain the whole range.
     * Where the runtime reports no range (not seen on ROCm 7.2), the weaker
     * check remains: the first and last bytes translate n - 1 apart, which
     * two registrations with a pageable gap between them can also pass. */
    char *a = (char *)pncxrt_host_dptr(p);
    if (a == nullptr || n == 0) return a;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&base, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) == hipSuccess &&
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) == hipSuccess &&
        base != nullptr && size > 0) {
        const char *lo = (const char *)base, *q = (const char *)p;
        return q >= lo && q + n <= lo + size ? a : nullptr;
    }
    (void)hipGetLastError();
    char *b = (char *)pncxrt_host_dptr((const char *)p + (n - 1));
    return b == a + (n - 1) ? a : nullptr;
}
void *pncxrt_host_dptr(const void *p) {
    /* the device address of pinned or registered host memory (the kernels
     * read and write it over PCIe), NULL for pageable or device memory */
    hipPointerAttribute_t at;
    void *d = nullptr;
    if (p == nullptr || hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost) return nullptr;
    if (hipHostGetDevicePointer(&d, (void *)p, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return d;
}
int pncxrt_ptr_device(const void *p) {
    hipPointerAttribute_t at;
    if (p == nullptr || hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return at.type == hipMemoryTypeDevice ? at.device : -1;
}
int pncxrt_is_device_ptr(const void *p) {
    /* device memory of the CURRENT device only: the kernels run there, and a
     * buffer on another GPU would fault without peer access (the file layer
     * refuses such a pointer: pncxrt_ptr_device) */
    const int d = pncxrt_ptr_device(p);
    int cur = -1;
    if (d < 0 || hipGetDevice(&cur) != hipSuccess) return 0;
    return d == cur;
}
}  // extern "C"
