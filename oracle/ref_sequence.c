/*
 * ref_sequence.c -- TEST INFRASTRUCTURE ONLY (bench.py's C1 cpu_baseline).
 *
 * The reference's single-rank C1 sequence for a same-type NC_INT request
 * (BASELINE configs[0]), restated with the oracle's swap on one thread and
 * timed in C, so the baseline carries no interpreter overhead:
 *   put = swap the user buffer in place, write the bytes at the variable's
 *         offset, swap the buffer back (ncmpio_getput.m4:186-214,269-270;
 *         the write is MPI-IO's pwrite on one rank);
 *   get = read the bytes into the user buffer, swap in place
 *         (ncmpio_getput.m4:415-470 -> ncmpio_unpack_xbuf,
 *         ncmpio_util.c:884-888).
 * Medians of `reps` calls in put_ms[0] / get_ms[0]; returns 0, or -1 on an
 * I/O error, -2 when the bytes read back differ from the ones written.
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
        err = read_all(fd, (char *)g, bytes, var_offset);
        orc_in_swapn(g, n, 4);
        tg[r] = now_ms() - t0;
    }
    if (!err && memcmp(g, h, bytes) != 0) err = -2;
    if (!err) {
        qsort(tp, (size_t)reps, sizeof(double), cmp_d);
        qsort(tg, (size_t)reps, sizeof(double), cmp_d);
        *put_ms = tp[reps / 2];
        *get_ms = tg[reps / 2];
    }
    if (fd >= 0) close(fd);
    free(h); free(g); free(tp); free(tg);
    return err;
}
