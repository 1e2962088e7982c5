/*
 * ref_sequence.c -- TEST INFRASTRUCTURE ONLY (bench.py's C1 cpu_baseline).
 *
 * The reference's single-rank C1 sequence for a same-type NC_INT request
 * (BASELINE configs[0]), restated with the oracle's swap on one thread and
 * timed in C, so the baseline carries no interpreter overhead:
 *   put = swap the user buffer in place, write the bytes at the variable's
 *         offset, swap the buffer back (ncmpio_getput.m4:186-214,269-270;
 *         the write is MPI-IO's pwrite on one rank);
 *   get = malloc a contiguous xbuf (a same-type get that needs a swap never
 *         reads into the user buffer: ncmpio_getput.m4:415-427), read the
 *         bytes into it, swap it in place, memcpy it into the user buffer,
 *         free it (ncmpio_unpack_xbuf, ncmpio_util.c:884-888,934-936;
 *         ncmpio_getput.m4:468-470).
 * Medians of `reps` calls in put_ms[0] / get_ms[0] (get_ms[1]: the older,
 * shorter restatement that reads straight into the user buffer and swaps
 * it, kept as a labelled second number); returns 0, or -1 on an I/O error,
 * -2 when the bytes read back differ from the ones written.
 *
 * orc_c1_first_sequence: the same calls under the reference's own
 * benchmark pattern (benchmarks/C/pnetcdf_put_vara.c:193-209), a record
 * variable whose records are each written once, appended past the end of
 * the file, then each read once.  A collective put of a record variable
 * also writes the grown numrecs into the header (ncmpio_getput.m4:272-311,
 * ncmpio_write_numrecs: 8 big-endian bytes at offset 4 in CDF-5).  The file
 * is cut back to `rec_offset` (its header) first.
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

void orc_in_swapn(void *buf, long long nelems, int esize);

static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec * 1e3 + (double)t.tv_nsec * 1e-6;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

static int write_all(int fd, const char *p, size_t n, long long off)
{
    while (n > 0) {
        const ssize_t w = pwrite(fd, p, n, (off_t)off);
        if (w <= 0) return -1;
        p += w; n -= (size_t)w; off += w;
    }
    return 0;
}

static int read_all(int fd, char *p, size_t n, long long off)
{
    while (n > 0) {
        const ssize_t r = pread(fd, p, n, (off_t)off);
        if (r <= 0) return -1;
        p += r; n -= (size_t)r; off += r;
    }
    return 0;
}

/* the reference's same-type get of n NC_INT at off into user: malloc xbuf,
 * read, swap in place, memcpy, free */
static int get_xbuf(int fd, uint32_t *user, long long n, long long off)
{
    const size_t bytes = (size_t)n * 4;
    void *x = malloc(bytes);
    int err;
    if (x == NULL) return -1;
    err = read_all(fd, (char *)x, bytes, off);
    if (!err) {
        orc_in_swapn(x, n, 4);
        memcpy(user, x, bytes);
    }
    free(x);
    return err;
}

int orc_c1_sequence(const char *path, long long var_offset, long long n, int reps, double *put_ms, double *get_ms)
{
    const size_t bytes = (size_t)n * 4;
    uint32_t *h = (uint32_t *)malloc(bytes), *g = (uint32_t *)malloc(bytes);
    double *tp = (double *)calloc((size_t)reps, sizeof(double)), *tg = (double *)calloc((size_t)reps, sizeof(double));
    int fd = open(path, O_RDWR), r, err = 0;
    long long i;
    if (!h || !g || !tp || !tg || fd < 0 || reps < 1) err = -1;
    for (i = 0; i < n && !err; i++) h[i] = (uint32_t)i * 2654435761u;
    for (r = 0; r < reps && !err; r++) {
        const double t0 = now_ms();
        orc_in_swapn(h, n, 4);
        err = write_all(fd, (const char *)h, bytes, var_offset);
        orc_in_swapn(h, n, 4);
        tp[r] = now_ms() - t0;
    }
    for (r = 0; r < reps && !err; r++) {
        const double t0 = now_ms();
        err = get_xbuf(fd, g, n, var_offset);
        tg[r] = now_ms() - t0;
    }
    if (!err && memcmp(g, h, bytes) != 0) err = -2;
    if (!err) {
        qsort(tp, (size_t)reps, sizeof(double), cmp_d);
        qsort(tg, (size_t)reps, sizeof(double), cmp_d);
        *put_ms = tp[reps / 2];
        get_ms[0] = tg[reps / 2];
    }
    for (r = 0; r < reps && !err; r++) {         /* the older restatement, labelled separately */
        const double t0 = now_ms();
        err = read_all(fd, (char *)g, bytes, var_offset);
        orc_in_swapn(g, n, 4);
        tg[r] = now_ms() - t0;
    }
    if (!err && memcmp(g, h, bytes) != 0) err = -2;
    if (!err) {
        qsort(tg, (size_t)reps, sizeof(double), cmp_d);
        get_ms[1] = tg[reps / 2];
    }
    if (fd >= 0) close(fd);
    free(h); free(g); free(tp); free(tg);
    return err;
}

/* out[0..5]: put median, get median, put min, get min (ms per call), the put
 * loop and the get loop (ms, all records) */
int orc_c1_first_sequence(const char *path, long long rec_offset, long long n, int nrec, double *out)
{
    const size_t bytes = (size_t)n * 4;
    uint32_t *h = (uint32_t *)malloc(bytes), *g = (uint32_t *)malloc(bytes);
    double *tp = (double *)calloc((size_t)nrec, sizeof(double)), *tg = (double *)calloc((size_t)nrec, sizeof(double));
    int fd = open(path, O_RDWR), r, err = 0;
    long long i;
    double loop;
    if (!h || !g || !tp || !tg || fd < 0 || nrec < 1) err = -1;
    if (!err && ftruncate(fd, (off_t)rec_offset) != 0) err = -1;
    for (i = 0; i < n && !err; i++) h[i] = (uint32_t)i * 2654435761u;
    loop = now_ms();
    for (r = 0; r < nrec && !err; r++) {
        unsigned char nr[8];
        const unsigned long long v = (unsigned long long)(r + 1);
        double t0;
        int b;
        for (i = 0; i < n; i++) h[i] += 1u;                 /* a new record's values (untimed) */
        t0 = now_ms();
        orc_in_swapn(h, n, 4);
        err = write_all(fd, (const char *)h, bytes, rec_offset + (long long)r * (long long)bytes);
        orc_in_swapn(h, n, 4);
        for (b = 0; b < 8; b++) nr[b] = (unsigned char)(v >> (56 - 8 * b));
        if (!err) err = write_all(fd, (const char *)nr, 8, 4);
        tp[r] = now_ms() - t0;
    }
    out[4] = now_ms() - loop;
    for (i = 0; i < n && !err; i++) h[i] -= (uint32_t)nrec;       /* record 0's values, less one */
    loop = 0;
    for (r = 0; r < nrec && !err; r++) {
        const double t0 = now_ms();
        err = get_xbuf(fd, g, n, rec_offset + (long long)r * (long long)bytes);
        tg[r] = now_ms() - t0;
        loop += tg[r];
        for (i = 0; i < n && !err; i++)
            if (g[i] != h[i] + (uint32_t)(r + 1)) err = -2;
    }
    out[5] = loop;
    if (!err) {
        qsort(tp, (size_t)nrec, sizeof(double), cmp_d);
        qsort(tg, (size_t)nrec, sizeof(double), cmp_d);
        out[0] = tp[nrec / 2];
        out[1] = tg[nrec / 2];
        out[2] = tp[0];
        out[3] = tg[0];
    }
    if (fd >= 0) close(fd);
    free(h); free(g); free(tp); free(tg);
    return err;
}
