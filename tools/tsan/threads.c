/*
 * ThreadSanitizer workload for the host code (file layer, I/O pool, staging,
 * warm-up thread), built and run on CPU by tools/tsan/run.sh.
 *
 * The reference tests six threads each creating, writing and reading its own
 * file (test/testcases/tst_pthread.c:175-227, 244-309); tests/mpi/api_check
 * pthread restates that on the GPU.  Here the same shape runs against a
 * synchronous CPU stand-in for the device (tools/tsan/cpudev_stub.c, byte
 * swaps only): NC_BYTE and NC_CHAR records (no conversion), NC_INT records
 * from host and from "device" buffers and NC_DOUBLE records, blocking and
 * nonblocking.  They go through everything the threads share: the file
 * table, the process-wide staging area and its lock, the per-device piece
 * events, the I/O pool (records of 2 MiB and more are cut into pool tasks),
 * the batch planner and its completion word, the create-time warm-up thread
 * and the enddef preload.  One more thread churns the file table with
 * header-only files and read-only reopens while the others write.
 *
 * Built against the no-device stub (tools/asan/pncxrt_stub.c) instead, it
 * runs the NC_BYTE / NC_CHAR paths only, without the staging lock between
 * the threads' first writes.
 *
 *   threads <dir> [nthreads] [iters]
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "pncx.h"
#include "pncx_nc.h"
#include "pncx_shim.h"

#define NX (2LL << 20)        /* one record: 2 MiB of NC_BYTE */
#define NI (1LL << 20)        /* one record: 2^20 NC_INT (4 MiB), 2^19 NC_DOUBLE */
#define NREC 4

/* cpudev_stub.c; absent in the no-device build (tools/asan/pncxrt_stub.c) */
void cpudev_counts(long long *swap, long long *batch, long long *done) __attribute__((weak));

static const char *g_dir;
static int g_iters;
static int g_nodev;            /* no device: the NC_BYTE / NC_CHAR paths only */
/* the writers start their first data calls together: a lazily initialised
 * global is then first touched by several threads with nothing ordering
 * them, which is what the sanitizer needs to see a race (a lock taken in
 * between, e.g. by a staggered create, would order the accesses) */
static pthread_barrier_t g_start;

#define CHECK(e)                                                                       \
    do {                                                                               \
        int err_ = (e);                                                                \
        if (err_ != 0) {                                                               \
            fprintf(stderr, "thread %d: %s:%d: %s -> %d\n", id, __FILE__, __LINE__, #e, err_); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

/* NC_INT records: 0 from a host buffer, 1 from a "device" buffer, 2 and 3
 * nonblocking; NC_DOUBLE records 0 blocking, 1 nonblocking; then read back
 * to host and to the device buffer */
static int ints_and_doubles(int id, int ncid, int vi, int vd, int *ibuf, int *iback, double *dbuf,
                            double *dback, void *dev)
{
    pncx_offset start[2] = {0, 0}, count[2] = {1, NI};
    int r, req[4], st[4];
    CHECK(pncx_nc_put_varm(ncid, vi, start, count, NULL, NULL, ibuf, PNCX_ITYPE_INT));
    memcpy(dev, ibuf + NI, NI * 4);
    start[0] = 1;
    CHECK(pncx_nc_put_varm_dev(ncid, vi, start, count, NULL, NULL, dev, PNCX_ITYPE_INT, NULL));
    for (r = 2; r < NREC; r++) {
        start[0] = r;
        CHECK(pncx_nc_iput_varm(ncid, vi, start, count, NULL, NULL, ibuf + r * NI, PNCX_ITYPE_INT, &req[r - 2]));
    }
    count[1] = NI / 2;
    start[0] = 0;
    CHECK(pncx_nc_put_varm(ncid, vd, start, count, NULL, NULL, dbuf, PNCX_ITYPE_DOUBLE));
    start[0] = 1;
    CHECK(pncx_nc_iput_varm(ncid, vd, start, count, NULL, NULL, dbuf + NI / 2, PNCX_ITYPE_DOUBLE, &req[2]));
    CHECK(pncx_nc_wait_all(ncid, 3, req, st));
    CHECK(st[0] | st[1] | st[2]);
    start[0] = 0;
    count[0] = NREC;
    count[1] = NI;
    memset(iback, 0, NI * NREC * 4);
    CHECK(pncx_nc_get_varm(ncid, vi, start, count, NULL, NULL, iback, PNCX_ITYPE_INT));
    count[0] = 2;
    count[1] = NI / 2;
    memset(dback, 0, NI * 8);
    CHECK(pncx_nc_get_varm(ncid, vd, start, count, NULL, NULL, dback, PNCX_ITYPE_DOUBLE));
    if (memcmp(iback, ibuf, NI * NREC * 4) != 0 || memcmp(dback, dbuf, NI * 8) != 0) {
        fprintf(stderr, "thread %d: int/double records differ\n", id);
        return 1;
    }
    start[0] = 3;
    count[0] = 1;
    count[1] = NI;
    memset(dev, 0, NI * 4);
    CHECK(pncx_nc_get_varm_dev(ncid, vi, start, count, NULL, NULL, dev, PNCX_ITYPE_INT, NULL));
    if (memcmp(dev, ibuf + 3 * NI, NI * 4) != 0) {
        fprintf(stderr, "thread %d: device-buffer get differs\n", id);
        return 1;
    }
    return 0;
}

#undef CHECK
#define CHECK(e)                                                                       \
    do {                                                                               \
        int err_ = (e);                                                                \
        if (err_ != 0) {                                                               \
            fprintf(stderr, "thread %d: %s:%d: %s -> %d\n", id, __FILE__, __LINE__, #e, err_); \
            return (void *)1;                                                          \
        }                                                                              \
    } while (0)

static void *writer(void *arg)
{
    const int id = (int)(long)arg;
    signed char *buf = malloc(NX * NREC), *back = malloc(NX * NREC);
    int *ibuf = malloc(NI * NREC * 4), *iback = malloc(NI * NREC * 4);
    double *dbuf = malloc(NI * 8), *dback = malloc(NI * 8);   /* two records of NI / 2 */
    void *dev = NULL;
    char path[512], title[64];
    int it, r;
    if (buf == NULL || back == NULL || ibuf == NULL || iback == NULL || dbuf == NULL || dback == NULL ||
        (!g_nodev && pncxrt_malloc(&dev, NI * 4) != 0))
        return (void *)1;
    for (it = 0; it < g_iters; it++) {
        int ncid, dt, dx, dims[2], vr, vc, vi, vd, req[NREC], st[NREC], err;
        pncx_offset start[2], count[2];
        snprintf(path, sizeof path, "%s/tsan_%d_%d.nc", g_dir, id, it);
        for (r = 0; r < NX * NREC; r++) buf[r] = (signed char)(r * 7 + id * 13 + it);
        for (r = 0; r < NI * NREC; r++) ibuf[r] = r * 31 - id * 1000003 + it;
        for (r = 0; r < NI; r++) dbuf[r] = r * 0.5 - id - it;
        CHECK(pncx_nc_create(path, NC_CLOBBER | NC_64BIT_DATA, &ncid));
        CHECK(pncx_nc_def_dim(ncid, "t", NC_UNLIMITED, &dt));
        CHECK(pncx_nc_def_dim(ncid, "x", NX, &dx));
        dims[0] = dt;
        dims[1] = dx;
        CHECK(pncx_nc_def_var(ncid, "r", NC_BYTE, 2, dims, &vr));
        CHECK(pncx_nc_def_var(ncid, "c", NC_CHAR, 1, &dx, &vc));
        CHECK(pncx_nc_def_dim(ncid, "xi", NI, &dims[1]));
        CHECK(pncx_nc_def_var(ncid, "i", NC_INT, 2, dims, &vi));
        CHECK(pncx_nc_def_dim(ncid, "xd", NI / 2, &dims[1]));
        CHECK(pncx_nc_def_var(ncid, "d", NC_DOUBLE, 2, dims, &vd));
        snprintf(title, sizeof title, "thread %d iteration %d", id, it);
        CHECK(pncx_nc_put_att(ncid, NC_GLOBAL, "title", NC_CHAR, (pncx_offset)strlen(title), title,
                              PNCX_ITYPE_CHAR));
        CHECK(pncx_nc_enddef(ncid));
        if (it == 0) pthread_barrier_wait(&g_start);
        /* records 0 and 1 blocking, 2 and 3 nonblocking */
        for (r = 0; r < 2; r++) {
            start[0] = r; start[1] = 0; count[0] = 1; count[1] = NX;
            CHECK(pncx_nc_put_varm(ncid, vr, start, count, NULL, NULL, buf + r * NX, PNCX_ITYPE_SCHAR));
        }
        for (r = 2; r < NREC; r++) {
            start[0] = r; start[1] = 0; count[0] = 1; count[1] = NX;
            CHECK(pncx_nc_iput_varm(ncid, vr, start, count, NULL, NULL, buf + r * NX, PNCX_ITYPE_SCHAR,
                                    &req[r - 2]));
        }
        CHECK(pncx_nc_wait_all(ncid, NREC - 2, req, st));
        CHECK(st[0] | st[1]);
        start[0] = 0; count[0] = NX;
        CHECK(pncx_nc_put_varm(ncid, vc, start, count, NULL, NULL, buf, PNCX_ITYPE_CHAR));
        memset(back, 0, NX * NREC);
        start[0] = 0; start[1] = 0; count[0] = NREC; count[1] = NX;
        CHECK(pncx_nc_get_varm(ncid, vr, start, count, NULL, NULL, back, PNCX_ITYPE_SCHAR));
        if (memcmp(back, buf, NX * NREC) != 0) {
            fprintf(stderr, "thread %d: records differ\n", id);
            return (void *)1;
        }
        if (!g_nodev && (err = ints_and_doubles(id, ncid, vi, vd, ibuf, iback, dbuf, dback, dev)) != 0)
            return (void *)1;
        CHECK(pncx_nc_close(ncid));
        /* read-only reopen: the records and the text variable */
        CHECK(pncx_nc_open(path, NC_NOWRITE, &ncid));
        memset(back, 0, NX * NREC);
        start[0] = 1; start[1] = 0; count[0] = 2; count[1] = NX;
        CHECK(pncx_nc_get_varm(ncid, vr, start, count, NULL, NULL, back, PNCX_ITYPE_SCHAR));
        start[0] = 0; count[0] = NX;
        CHECK(pncx_nc_get_varm(ncid, vc, start, count, NULL, NULL, back + 2 * NX, PNCX_ITYPE_CHAR));
        if (memcmp(back, buf + NX, 2 * NX) != 0 || memcmp(back + 2 * NX, buf, NX) != 0) {
            fprintf(stderr, "thread %d: reopened file differs\n", id);
            return (void *)1;
        }
        CHECK(pncx_nc_close(ncid));
        unlink(path);
    }
    free(buf);
    free(back);
    free(ibuf);
    free(iback);
    free(dbuf);
    free(dback);
    pncxrt_free(dev);
    return NULL;
}

/* header-only files and reopens while the writers run */
static void *churn(void *arg)
{
    const int id = (int)(long)arg;
    char path[512];
    int it;
    for (it = 0; it < 8 * g_iters; it++) {
        int ncid, dx, v, nd, nv, ng, ul;
        snprintf(path, sizeof path, "%s/tsan_churn_%d.nc", g_dir, it % 3);
        CHECK(pncx_nc_create(path, NC_CLOBBER, &ncid));
        CHECK(pncx_nc_def_dim(ncid, "x", 10 + it, &dx));
        CHECK(pncx_nc_def_var(ncid, "v", NC_BYTE, 1, &dx, &v));
        CHECK(pncx_nc_close(ncid));
        CHECK(pncx_nc_open(path, NC_NOWRITE, &ncid));
        CHECK(pncx_nc_inq(ncid, &nd, &nv, &ng, &ul));
        if (nd != 1 || nv != 1) return (void *)1;
        CHECK(pncx_nc_close(ncid));
    }
    for (it = 0; it < 3; it++) {
        snprintf(path, sizeof path, "%s/tsan_churn_%d.nc", g_dir, it);
        unlink(path);
    }
    return NULL;
}

int main(int argc, char **argv)
{
    int n, i, bad = 0;
    pthread_t th[65];
    if (argc < 2) {
        fprintf(stderr, "usage: threads <dir> [nthreads] [iters]\n");
        return 2;
    }
    g_dir = argv[1];
    n = argc > 2 ? atoi(argv[2]) : 6;
    g_iters = argc > 3 ? atoi(argv[3]) : 3;
    g_nodev = cpudev_counts == NULL;
    if (n < 1 || n > 64 || g_iters < 1) return 2;
    pthread_barrier_init(&g_start, NULL, (unsigned)n);
    for (i = 0; i < n; i++) pthread_create(&th[i], NULL, writer, (void *)(long)i);
    pthread_create(&th[n], NULL, churn, (void *)(long)n);
    for (i = 0; i <= n; i++) {
        void *rv;
        pthread_join(th[i], &rv);
        bad += rv != NULL;
    }
    if (bad) {
        fprintf(stderr, "%d thread(s) failed\n", bad);
        return 1;
    }
    if (g_nodev) {
        printf("threads ok %d writers x %d files + churn; no device\n", n, g_iters);
        return 0;
    }
    {
        long long ns, nb, nd;
        cpudev_counts(&ns, &nb, &nd);
        printf("threads ok %d writers x %d files + churn; device stand-in: %lld swap, %lld batch, %lld completion "
               "launches\n", n, g_iters, ns, nb, nd);
        if (ns == 0 || nb == 0 || nd == 0) return 1;     /* the device paths must have run */
    }
    return 0;
}
