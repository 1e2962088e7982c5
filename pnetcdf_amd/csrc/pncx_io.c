/*
 * pncx_io.c -- parallel POSIX I/O pool (see pncx_io.h).
 *
 * The reference hands the packed buffer to MPI-IO (ncmpio_file_io.c); for one
 * process on a node-local file system the cost is the page-cache copy, which
 * one thread does at a few GB/s.  Splitting the copy over the host cores the
 * box gives a GPU (PNCX_IO_THREADS, default 8) raises that, and running it
 * asynchronously lets it overlap the GPU conversion of the next chunk.
 *
 * Writes: pwrite into one file serialises on the inode lock, so more threads
 * do not help (measured on tmpfs: 4.8 GB/s with 1 thread, 4.3 with 8).
 * Copies into a shared mapping of the file do scale (49 GB/s with 8
 * threads, 4 GB/s on first touch vs 2 for pwrite).  Large write runs
 * therefore go through mmap + memcpy: the pool first grows the file with
 * fallocate (never shrinks it, so ranks writing disjoint records of one file
 * stay safe), then each task maps its page-aligned window.  Runs under
 * MMAP_MIN bytes (unless many of them fill a span densely: one mapping per
 * share then), file systems without fallocate and PNCX_IO_MMAP=0 use
 * pwrite.  Reads use pread, which takes the shared lock and scales.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "pncx.h"
#include "pncx_nc.h"
#include "pncx_io.h"
#include "pncx_shim.h"

#define MAX_THREADS 64
#define INLINE_BYTES (1u << 20)      /* below this a job runs in the caller */
#define MIN_TASK_BYTES (1u << 20)    /* no task smaller than this */
#define MMAP_MIN (256u << 10)        /* smallest write run copied through a mapping */

typedef struct task {
    struct task *next;
    pio_batch *b;
    int fd, write;                   /* write: 1 = pwrite, 2 = mmap + memcpy for large runs,
                                      * 3 = one mapping per share over many small runs */
    pio_run *runs;                   /* shared by the tasks of one job */
    size_t n;
    long long lo, hi;                /* byte range of the concatenated runs */
    int *refs;                       /* tasks still using runs[] */
} task;

static pthread_mutex_t q_lock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t q_cond = PTHREAD_COND_INITIALIZER;
static task *q_head, *q_tail;
static int n_threads = -1;

int pio_write_all(int fd, const void *buf, size_t n, long long off)
{
    const char *p = (const char *)buf;
    while (n > 0) {
        const size_t m = n > (1u << 30) ? (1u << 30) : n;
        const ssize_t w = pwrite(fd, p, m, (off_t)off);
        if (w < 0) { if (errno == EINTR) continue; return NC_EWRITE; }
        if (w == 0) return NC_EWRITE;
        p += w; n -= (size_t)w; off += w;
    }
    return NC_NOERR;
}

/* reads past the end of file return zeros (never-written data) */
int pio_read_all(int fd, void *buf, size_t n, long long off)
{
    char *p = (char *)buf;
    while (n > 0) {
        const size_t m = n > (1u << 30) ? (1u << 30) : n;
        const ssize_t r = pread(fd, p, m, (off_t)off);
        if (r < 0) { if (errno == EINTR) continue; return NC_EREAD; }
        if (r == 0) { memset(p, 0, n); return NC_NOERR; }
        p += r; n -= (size_t)r; off += r;
    }
    return NC_NOERR;
}

static long g_page;

/* MAP_POPULATE enters a mapping's pages in one pass instead of one fault
 * each: 4 MiB on one thread 174 us against 514 (tools/c1_probe.hip), but a
 * 1 GiB put over 8 mapped tasks ran at 18.7 GiB/s with it and 22.3 without
 * (profiles/r04j_host_modes.txt), and single writers now use pwrite.  Off
 * by default; PNCX_IO_POPULATE=1 turns it on (A/B). */
static int populate(void)
{
    return pncx_knob(PNCXK_KNOB_IO_POPULATE) == 1 ? MAP_POPULATE : 0;
}

/* memcpy into a shared mapping of the file (the range lies inside the file) */
static int map_write(int fd, const unsigned char *src, size_t n, long long off)
{
    const long long base = off - off % g_page;
    const size_t span = (size_t)(off - base) + n;
    unsigned char *m = (unsigned char *)mmap(NULL, span, PROT_WRITE, MAP_SHARED | populate(), fd, (off_t)base);
    if (m == MAP_FAILED) return pio_write_all(fd, src, n, off);
    memcpy(m + (off - base), src, n);
    munmap(m, span);
    return NC_NOERR;
}

/* Many small write runs (e.g. the rows of a rank's subarray): one mapping
 * over the file span of this share, then a memcpy per run.  pwrite of 8 KiB
 * rows took ~2 us each and serialised the ranks writing one file on the
 * inode lock (the reference's benchmarks/C/pnetcdf_put_vara.c, 4 ranks:
 * 1 GiB/s).  Returns 1 when the span is too sparse to map (caller pwrites). */
static int span_write(int fd, const pio_run *runs, size_t n, long long lo, long long hi)
{
    long long pos = 0, fmin = -1, fmax = 0, bytes = hi - lo, base;
    size_t i, span;
    unsigned char *m;
    for (i = 0; i < n && pos < hi; i++) {
        const long long a = pos, b = pos + runs[i].len;
        pos = b;
        if (b <= lo) continue;
        {
            const long long s = a > lo ? a : lo, e = b < hi ? b : hi, k = s - a;
            if (fmin < 0 || runs[i].off + k < fmin) fmin = runs[i].off + k;
            if (runs[i].off + k + (e - s) > fmax) fmax = runs[i].off + k + (e - s);
        }
    }
    if (fmin < 0) return 0;
    if (fmax - fmin > 4 * bytes) return 1;
    base = fmin - fmin % g_page;
    span = (size_t)(fmax - base);
    m = (unsigned char *)mmap(NULL, span, PROT_WRITE, MAP_SHARED | populate(), fd, (off_t)base);
    if (m == MAP_FAILED) return 1;
    for (i = 0, pos = 0; i < n && pos < hi; i++) {
        const long long a = pos, b = pos + runs[i].len;
        pos = b;
        if (b <= lo) continue;
        {
            const long long s = a > lo ? a : lo, e = b < hi ? b : hi, k = s - a;
            memcpy(m + (runs[i].off + k - base), runs[i].mem + k, (size_t)(e - s));
        }
    }
    munmap(m, span);
    return 0;
}

/* copy bytes [lo, hi) of the concatenation of runs */
static int do_range(int fd, int write, const pio_run *runs, size_t n, long long lo, long long hi)
{
    long long pos = 0;
    size_t i;
    int err = NC_NOERR;
    if (write == 3) {
        if (span_write(fd, runs, n, lo, hi) == 0) return NC_NOERR;
        write = 1;
    }
    for (i = 0; i < n && pos < hi && !err; i++) {
        const long long a = pos, b = pos + runs[i].len;
        pos = b;
        if (b <= lo) continue;
        {
            const long long s = a > lo ? a : lo, e = b < hi ? b : hi;
            const long long k = s - a;
            if (!write)
                err = pio_read_all(fd, runs[i].mem + k, (size_t)(e - s), runs[i].off + k);
            else if (write == 2 && e - s >= (long long)MMAP_MIN)
                err = map_write(fd, runs[i].mem + k, (size_t)(e - s), runs[i].off + k);
            else
                err = pio_write_all(fd, runs[i].mem + k, (size_t)(e - s), runs[i].off + k);
        }
    }
    return err;
}

/* read once per process; every thread sees g_page set before the mode
 * (a thread that found the mode set with g_page still 0 would divide by it) */
static int g_mmap_mode;
static pthread_once_t g_mmap_once = PTHREAD_ONCE_INIT;
static void mmap_mode_init(void)
{
    const char *e = getenv("PNCX_IO_MMAP");
    g_page = sysconf(_SC_PAGESIZE);
    if (g_page <= 0) g_page = 4096;
    g_mmap_mode = e ? atoi(e) != 0 : 1;
}

static int mmap_mode(void)
{
    pthread_once(&g_mmap_once, mmap_mode_init);
    return g_mmap_mode;
}

/* Write job through mappings?  Large runs (>= MMAP_MIN) are each mapped;
 * a job of small runs whose file span is at most 4x its bytes is mapped one
 * span per share.  The file must already cover what is mapped: grow it with
 * fallocate where needed (a mapping cannot extend a file). */
static int write_mode(int fd, const pio_run *runs, size_t n, long long total)
{
    struct stat st;
    long long end = 0, fmin = -1, fmax = 0;
    size_t i;
    int mode = 2;
    if (!mmap_mode() || total < (long long)MMAP_MIN) return 1;
    for (i = 0; i < n; i++) {
        if (runs[i].len >= (long long)MMAP_MIN && runs[i].off + runs[i].len > end) end = runs[i].off + runs[i].len;
        if (runs[i].len > 0 && (fmin < 0 || runs[i].off < fmin)) fmin = runs[i].off;
        if (runs[i].off + runs[i].len > fmax) fmax = runs[i].off + runs[i].len;
    }
    if (end == 0) {
        if (fmin < 0 || fmax - fmin > 4 * total) return 1;
        end = fmax;
        mode = 3;
    }
    if (fstat(fd, &st) != 0) return 1;
    if (end > (long long)st.st_size &&
        fallocate(fd, 0, (off_t)st.st_size, (off_t)(end - (long long)st.st_size)) != 0)
        return 1;
    return mode;
}

/* one share of a job is done: record its error, release the shared runs */
static void share_done(pio_batch *b, pio_run *runs, int *refs, int err)
{
    int last;
    pthread_mutex_lock(&b->m);
    if (err && !b->err) b->err = err;
    b->pending--;
    if (b->pending == 0) pthread_cond_broadcast(&b->c);
    pthread_mutex_unlock(&b->m);
    pthread_mutex_lock(&q_lock);
    last = --(*refs) == 0;
    pthread_mutex_unlock(&q_lock);
    if (last) { free(runs); free(refs); }
}

static void finish(task *t, int err)
{
    share_done(t->b, t->runs, t->refs, err);
    free(t);
}

static void *worker(void *arg)
{
    (void)arg;
    for (;;) {
        task *t;
        pthread_mutex_lock(&q_lock);
        while (q_head == NULL) pthread_cond_wait(&q_cond, &q_lock);
        t = q_head;
        q_head = t->next;
        if (q_head == NULL) q_tail = NULL;
        pthread_mutex_unlock(&q_lock);
        finish(t, do_range(t->fd, t->write, t->runs, t->n, t->lo, t->hi));
    }
    return NULL;
}

int pio_threads(void)
{
    pthread_mutex_lock(&q_lock);
    if (n_threads < 0) {
        const char *e = getenv("PNCX_IO_THREADS");
        int n = e ? atoi(e) : 8, i;
        if (n < 1) n = 1;
        if (n > MAX_THREADS) n = MAX_THREADS;
        n_threads = 0;
        for (i = 0; i < n; i++) {
            pthread_t th;
            pthread_attr_t at;
            pthread_attr_init(&at);
            pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
            if (pthread_create(&th, &at, worker, NULL) == 0) n_threads++;
            pthread_attr_destroy(&at);
        }
    }
    pthread_mutex_unlock(&q_lock);
    return n_threads;
}

void pio_batch_init(pio_batch *b)
{
    pthread_mutex_init(&b->m, NULL);
    pthread_cond_init(&b->c, NULL);
    b->pending = 0;
    b->err = NC_NOERR;
}

void pio_batch_destroy(pio_batch *b)
{
    pthread_mutex_destroy(&b->m);
    pthread_cond_destroy(&b->c);
}

/* queue the job as nt tasks of about equal byte ranges */
static int queue_tasks(pio_batch *b, int fd, int write, const pio_run *runs, size_t n, long long total, int nt)
{
    long long per;
    int k, *refs;
    pio_run *copy;
    copy = (pio_run *)malloc(sizeof(pio_run) * n);
    refs = (int *)malloc(sizeof(int));
    if (copy == NULL || refs == NULL) { free(copy); free(refs); return NC_ENOMEM; }
    memcpy(copy, runs, sizeof(pio_run) * n);
    *refs = nt;
    per = (total + nt - 1) / nt;
    pthread_mutex_lock(&b->m);
    b->pending += nt;
    pthread_mutex_unlock(&b->m);
    for (k = 0; k < nt; k++) {
        task *t = (task *)calloc(1, sizeof(task));
        const long long lo = k * per, hi = (k + 1) * per < total ? (k + 1) * per : total;
        if (t == NULL) {                     /* no memory for a task: run this share inline */
            share_done(b, copy, refs, do_range(fd, write, copy, n, lo, hi));
            continue;
        }
        t->b = b;
        t->fd = fd;
        t->write = write;
        t->runs = copy;
        t->n = n;
        t->lo = lo;
        t->hi = hi;
        t->refs = refs;
        pthread_mutex_lock(&q_lock);
        if (q_tail) q_tail->next = t; else q_head = t;
        q_tail = t;
        pthread_cond_signal(&q_cond);
        pthread_mutex_unlock(&q_lock);
    }
    return NC_NOERR;
}

int pio_submit(pio_batch *b, int fd, int write, const pio_run *runs, size_t n)
{
    long long total = 0;
    size_t i;
    int nt, tasks;
    for (i = 0; i < n; i++) total += runs[i].len;
    if (total == 0) return NC_NOERR;
    nt = total < INLINE_BYTES ? 0 : pio_threads();
    tasks = nt;
    if ((long long)tasks * MIN_TASK_BYTES > total) tasks = (int)(total / MIN_TASK_BYTES);
    if (tasks < 1) tasks = 1;
    /* one writer: pwrite (4 MiB on the MI355X host: 108 us, against 514 us
     * through a mapping and 174 us with MAP_POPULATE, tools/c1_probe.hip);
     * mappings only when several tasks write one file at once */
    if (write) write = (nt <= 1 || tasks <= 1) ? 1 : write_mode(fd, runs, n, total);
    if (nt <= 1) {
        const int err = do_range(fd, write, runs, n, 0, total);
        if (err) {
            pthread_mutex_lock(&b->m);
            if (!b->err) b->err = err;
            pthread_mutex_unlock(&b->m);
        }
        return err;
    }
    return queue_tasks(b, fd, write, runs, n, total, tasks);
}

/* Reads of a small job spread over `parts` pool threads (pread of one
 * tmpfs file takes no exclusive lock, so the copies run side by side);
 * pieces of at least 64 KiB. */
int pio_read_split(pio_batch *b, int fd, const pio_run *runs, size_t n, int parts)
{
    long long total = 0;
    size_t i;
    int nt = pio_threads();
    for (i = 0; i < n; i++) total += runs[i].len;
    if (total == 0) return NC_NOERR;
    if (parts > nt) parts = nt;
    if ((long long)parts * (64 << 10) > total) parts = (int)(total / (64 << 10));
    if (parts < 2) {
        const int err = do_range(fd, 0, runs, n, 0, total);
        if (err) {
            pthread_mutex_lock(&b->m);
            if (!b->err) b->err = err;
            pthread_mutex_unlock(&b->m);
        }
        return err;
    }
    return queue_tasks(b, fd, 0, runs, n, total, parts);
}

int pio_wait(pio_batch *b)
{
    int err;
    pthread_mutex_lock(&b->m);
    while (b->pending > 0) pthread_cond_wait(&b->c, &b->m);
    err = b->err;
    b->err = NC_NOERR;
    pthread_mutex_unlock(&b->m);
    return err;
}

int pio_rw_inline(int fd, int write, const pio_run *runs, size_t n)
{
    long long total = 0;
    size_t i;
    for (i = 0; i < n; i++) total += runs[i].len;
    return total == 0 ? NC_NOERR : do_range(fd, write ? 1 : 0, runs, n, 0, total);
}

int pio_rw(int fd, int write, const pio_run *runs, size_t n)
{
    pio_batch b;
    int err, e2;
    pio_batch_init(&b);
    err = pio_submit(&b, fd, write, runs, n);
    e2 = pio_wait(&b);
    pio_batch_destroy(&b);
    return err ? err : e2;
}
