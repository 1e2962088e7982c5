/*
 * api_check.c -- programs written against the public ncmpi_* API
 * (include/pnetcdf.h) and linked with libpnetcdf.so, in the shape of the
 * reference's benchmarks and tests.  Test infrastructure: tests/
 * test_gpu_c_api.py and tests/test_c_api_cpu.py run the modes and check
 * the files they write against the CPU oracle.
 *
 *   api_check c1 <nc> <in.bin> <n> [dev]
 *       BASELINE config 1 (benchmarks/C pattern, 1 rank): 1-D NC_INT x(n),
 *       ncmpi_put_vara_int_all of in.bin, close, reopen,
 *       ncmpi_get_vara_int_all (must equal the input) and
 *       ncmpi_get_vara_double_all (config 3's read: must equal (double)).
 *       dev = 1: the user buffers are hipMalloc'ed (device-resident path).
 *   api_check c1bench <nc> <n> <reps> <dev>
 *       config 1 timed: reps x ncmpi_put_vara_int_all, then reps x
 *       ncmpi_get_vara_int_all of 1-D NC_INT x(n) on one open file (host or
 *       hipMalloc'ed buffers); prints median/min ms and the variable's offset.
 *   api_check c1first <nc> <n> <nrec> <dev> [double]
 *       config 1 under benchmarks/C/pnetcdf_put_vara.c's pattern: a record
 *       variable x(time, n) NC_INT, each record put once (appended), then
 *       each record got once; per-call medians, loop and close times.
 *       double: through ncmpi_put/get_vara_double_all (cross-type).
 *   api_check c1ab <nc> <n> <nrec> <knob> <a> <b> [dev]
 *       c1first with a libpncx knob alternating between a and b record by
 *       record: put and get medians under each value (A/B in one process).
 *   api_check numrecs <nc>
 *       on N ranks: collective record puts must leave numrecs in the FILE
 *       (ncmpio_getput.m4:272-311), fixed-size puts must not touch it; rank
 *       0 reads the header's numrecs bytes after every put.
 *   api_check openfail <dir>
 *       on 2+ ranks: with a file open, an open and a create that fail on
 *       the last rank only must leave the open file usable everywhere, and
 *       the failed create must remove its file.
 *   api_check bputshort <nc>
 *       bput_vara with a predefined buftype and a bufcount short of the
 *       request: NC_EIOMISMATCH (ncmpio_i_getput.m4:216).
 *   api_check putvara <nc> <nvars> <len> <ntimes> <nonblocking> [indep]
 *       benchmarks/C/pnetcdf_put_vara.c:138-219 on 1..N ranks: record
 *       variables float var_i(time, Y, X), text/float/short attributes,
 *       ncmpi_iput_vara_float x nvars x ntimes + ncmpi_wait_all (or
 *       ncmpi_put_vara_float[_all]); each rank a 2-D block.
 *   api_check c4 <nc> <shorts.bin> <floats.bin> <nel> <erange> [dev]
 *       BASELINE config 4: 256 variables, ncmpi_iput_vara_short/float x 256
 *       + one ncmpi_wait_all; erange = 1 is §8(d)'s secondary variant (the
 *       NC_SHORT variables written from float with NC_ERANGE).  dev = 1:
 *       the 256 user buffers are hipMalloc'ed.
 *   api_check records <nc> <nrec> <x>
 *       config 5 at file level on N ranks: a record variable
 *       v(time, x) NC_DOUBLE, rank r writes its slab of records with
 *       ncmpi_put_vara_double_all; reopened, every rank reads every record.
 *   api_check errors <dir>
 *       argument and mode errors the dispatcher returns before any
 *       conversion (no GPU needed): prints "name code" lines.
 *   api_check header <nc> [nranks-agnostic]
 *       define-mode only (dims, variables, text attributes) on N ranks: the
 *       header rank 0 writes must not depend on N.
 *   api_check pthread <prefix> <nthreads> <nx> <ny> <coll> [dev]
 *       test/testcases/tst_pthread.c:38,145-309 restated: nthreads threads
 *       (MPI_THREAD_MULTIPLE), each on its own file <prefix>.<id> over
 *       MPI_COMM_SELF: a record variable ivar(time, X) NC_INT and a fixed
 *       dvar(Y, X) NC_DOUBLE; records 0 and 2 of ivar with
 *       ncmpi_put_vara_int[_all], dvar with ncmpi_put_var_double[_all],
 *       sync, close; after a barrier of the threads each thread opens the
 *       file of thread id+1, reads both records and dvar back and checks
 *       them.  Values: ivar record r element i = id*1000003 + r*7919 + i,
 *       dvar element i = id + i*0.5.  dev = 1: hipMalloc'ed buffers.
 *       One JSON line per thread: the variables' offsets, recsize, errors.
 *   api_check pthreadhdr <prefix> <nthreads> <iters>
 *       define-mode only, no GPU: each thread creates / defines / closes /
 *       reopens / inquires / closes its own file iters times; no file may
 *       stay open at the end (the ncid table under threads).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <mpi.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pnetcdf.h"

static int nerrs = 0;
#define CHECK(call)                                                                                  \
    do {                                                                                             \
        int _e = (call);                                                                             \
        if (_e != NC_NOERR) {                                                                        \
            fprintf(stderr, "%s:%d: %s -> %d %s\n", __FILE__, __LINE__, #call, _e, ncmpi_strerror(_e)); \
            nerrs++;                                                                                 \
        }                                                                                            \
    } while (0)

static void *slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    void *b;
    if (f == NULL) return NULL;
    fseek(f, 0, SEEK_END);
    *len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    b = malloc(*len + 1);
    if (b && fread(b, 1, *len, f) != *len) { free(b); b = NULL; }
    fclose(f);
    return b;
}

/* device copies of host data (hipMalloc), for the device-resident variants */
static void *to_dev(const void *h, size_t n)
{
    void *d = NULL;
    if (hipMalloc(&d, n ? n : 1) != hipSuccess) { fprintf(stderr, "hipMalloc failed\n"); exit(3); }
    if (n && h && hipMemcpy(d, h, n, hipMemcpyHostToDevice) != hipSuccess) { fprintf(stderr, "H2D failed\n"); exit(3); }
    return d;
}
static void from_dev(void *h, const void *d, size_t n)
{
    if (hipMemcpy(h, d, n, hipMemcpyDeviceToHost) != hipSuccess) { fprintf(stderr, "D2H failed\n"); exit(3); }
}

static int mode_c1(const char *path, const char *inpath, MPI_Offset n, int dev)
{
    size_t len;
    int *in = (int *)slurp(inpath, &len), *got, ncid, dimid, varid, i;
    double *gd;
    void *din = NULL, *dgot = NULL, *dgd = NULL;
    MPI_Offset start[1] = {0}, count[1] = {n}, put = 0, get = 0;
    if (in == NULL || len != (size_t)n * 4) { fprintf(stderr, "bad input\n"); return 1; }
    got = (int *)calloc((size_t)n, sizeof(int));
    gd = (double *)calloc((size_t)n, sizeof(double));
    if (dev) {
        din = to_dev(in, (size_t)n * 4);
        dgot = to_dev(NULL, (size_t)n * 4);
        dgd = to_dev(NULL, (size_t)n * 8);
    }
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "x", n, &dimid));
    CHECK(ncmpi_def_var(ncid, "v", NC_INT, 1, &dimid, &varid));
    CHECK(ncmpi_enddef(ncid));
    CHECK(ncmpi_put_vara_int_all(ncid, varid, start, count, dev ? din : (void *)in));
    CHECK(ncmpi_inq_put_size(ncid, &put));
    CHECK(ncmpi_close(ncid));
    CHECK(ncmpi_open(MPI_COMM_WORLD, path, NC_NOWRITE, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_inq_varid(ncid, "v", &varid));
    CHECK(ncmpi_get_vara_int_all(ncid, varid, start, count, dev ? dgot : (void *)got));
    CHECK(ncmpi_get_vara_double_all(ncid, varid, start, count, dev ? dgd : (void *)gd));
    CHECK(ncmpi_inq_get_size(ncid, &get));
    CHECK(ncmpi_close(ncid));
    if (dev) {
        from_dev(got, dgot, (size_t)n * 4);
        from_dev(gd, dgd, (size_t)n * 8);
        hipFree(din);
        hipFree(dgot);
        hipFree(dgd);
    }
    for (i = 0; i < n; i++) {
        if (got[i] != in[i]) { fprintf(stderr, "int mismatch at %d\n", i); nerrs++; break; }
        if (gd[i] != (double)in[i]) { fprintf(stderr, "double mismatch at %d\n", i); nerrs++; break; }
    }
    printf("{\"mode\": \"c1\", \"n\": %lld, \"put_size\": %lld, \"get_size\": %lld, \"errors\": %d}\n",
           (long long)n, (long long)put, (long long)get, nerrs);
    free(in);
    free(got);
    free(gd);
    return nerrs != 0;
}

/* benchmarks/C/pnetcdf_put_vara.c:90-219 restated as a check */
static int mode_putvara(const char *path, int nvars, int len, int ntimes, int nonblocking, int indep)
{
    int i, j, rank, nprocs, psizes[2] = {0, 0}, ncid, *varid, dimid[3];
    float **buf;
    MPI_Offset start[3], count[3];
    double t0, t1, tmax;
    char name[64], str_att[128];
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
    MPI_Dims_create(nprocs, 2, psizes);
    buf = (float **)malloc(sizeof(float *) * (size_t)nvars);
    varid = (int *)malloc(sizeof(int) * (size_t)nvars);
    for (i = 0; i < nvars; i++) {
        buf[i] = (float *)malloc(sizeof(float) * (size_t)len * (size_t)len);
        for (j = 0; j < len * len; j++) buf[i][j] = (float)(rank + i * len + j);
    }
    MPI_Barrier(MPI_COMM_WORLD);
    t0 = MPI_Wtime();
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    snprintf(str_att, sizeof str_att, "Thu Aug 29 14:29:35 2024");
    CHECK(ncmpi_put_att_text(ncid, NC_GLOBAL, "history", (MPI_Offset)strlen(str_att), str_att));
    CHECK(ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &dimid[0]));
    CHECK(ncmpi_def_dim(ncid, "Y", (MPI_Offset)psizes[0] * len, &dimid[1]));
    CHECK(ncmpi_def_dim(ncid, "X", (MPI_Offset)psizes[1] * len, &dimid[2]));
    for (i = 0; i < nvars; i++) {
        short short_att = 1234;
        float float_att[4] = {0, 1, 2, 3};
        snprintf(name, sizeof name, "var_%d", i);
        CHECK(ncmpi_def_var(ncid, name, NC_FLOAT, 3, dimid, &varid[i]));
        snprintf(str_att, sizeof str_att, "some text attribute %d type text.", i);
        CHECK(ncmpi_put_att_text(ncid, varid[i], "str_att", (MPI_Offset)strlen(str_att), str_att));
        CHECK(ncmpi_put_att_float(ncid, varid[i], "float_att", NC_FLOAT, 4, float_att));
        CHECK(ncmpi_put_att_short(ncid, varid[i], "short_att", NC_SHORT, 1, &short_att));
    }
    CHECK(ncmpi_enddef(ncid));
    if (indep) CHECK(ncmpi_begin_indep_data(ncid));
    start[1] = (MPI_Offset)len * (rank / psizes[1]);
    start[2] = (MPI_Offset)len * (rank % psizes[1]);
    count[0] = 1;
    count[1] = len;
    count[2] = len;
    t1 = MPI_Wtime();
    for (j = 0; j < ntimes; j++) {
        start[0] = j;
        for (i = 0; i < nvars; i++) {
            if (nonblocking) CHECK(ncmpi_iput_vara_float(ncid, varid[i], start, count, buf[i], NULL));
            else if (indep) CHECK(ncmpi_put_vara_float(ncid, varid[i], start, count, buf[i]));
            else CHECK(ncmpi_put_vara_float_all(ncid, varid[i], start, count, buf[i]));
        }
    }
    if (nonblocking) {
        if (indep) CHECK(ncmpi_wait(ncid, NC_REQ_ALL, NULL, NULL));
        else CHECK(ncmpi_wait_all(ncid, NC_REQ_ALL, NULL, NULL));
    }
    t1 = MPI_Wtime() - t1;
    if (indep) CHECK(ncmpi_end_indep_data(ncid));
    CHECK(ncmpi_close(ncid));
    t0 = MPI_Wtime() - t0;
    MPI_Reduce(&t1, &tmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    MPI_Allreduce(MPI_IN_PLACE, &nerrs, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (rank == 0) {
        const double w = 4.0 * nprocs * (double)len * len * nvars * ntimes;
        printf("{\"mode\": \"putvara\", \"nprocs\": %d, \"py\": %d, \"px\": %d, \"bytes\": %.0f, "
               "\"write_s\": %.6f, \"MiBps\": %.2f, \"errors\": %d}\n",
               nprocs, psizes[0], psizes[1], w, tmax, w / 1048576.0 / tmax, nerrs);
    }
    for (i = 0; i < nvars; i++) free(buf[i]);
    free(buf);
    free(varid);
    return nerrs != 0;
}

static int mode_c4(const char *path, const char *sp, const char *fp, MPI_Offset nel, int erange, int dev)
{
    const int nvar = 256;
    size_t ls, lf;
    short *sh = (short *)slurp(sp, &ls), *hsh = NULL;
    float *fl = (float *)slurp(fp, &lf), *hfl = NULL;
    int ncid, dimid, v, varid[256], reqs[256], st[256], err;
    MPI_Offset start[1] = {0}, count[1] = {nel};
    if (sh == NULL || fl == NULL || ls != (size_t)(nvar / 2) * nel * 2 || lf != (size_t)(nvar / 2) * nel * 4) {
        fprintf(stderr, "bad input\n");
        return 1;
    }
    if (dev) {                 /* the user buffers in HBM */
        hsh = sh;
        hfl = fl;
        sh = (short *)to_dev(hsh, ls);
        fl = (float *)to_dev(hfl, lf);
    }
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "x", nel, &dimid));
    for (v = 0; v < nvar; v++) {
        char name[32];
        snprintf(name, sizeof name, "v%d", v);
        CHECK(ncmpi_def_var(ncid, name, v % 2 == 0 ? NC_SHORT : NC_FLOAT, 1, &dimid, &varid[v]));
    }
    CHECK(ncmpi_enddef(ncid));
    for (v = 0; v < nvar; v++) {
        const MPI_Offset k = v / 2;
        if (v % 2 == 0 && !erange) CHECK(ncmpi_iput_vara_short(ncid, varid[v], start, count, sh + k * nel, &reqs[v]));
        else CHECK(ncmpi_iput_vara_float(ncid, varid[v], start, count, fl + k * nel, &reqs[v]));
    }
    err = ncmpi_wait_all(ncid, nvar, reqs, st);
    CHECK(ncmpi_close(ncid));
    printf("{\"mode\": \"c4\", \"wait\": %d, \"statuses\": [", err);
    for (v = 0; v < nvar; v++) printf("%s%d", v ? ", " : "", st[v]);
    printf("], \"reqs_after\": %d, \"errors\": %d}\n", reqs[0], nerrs);
    if (dev) {
        hipFree(sh);
        hipFree(fl);
        sh = hsh;
        fl = hfl;
    }
    free(sh);
    free(fl);
    return nerrs != 0;
}

static int mode_records(const char *path, MPI_Offset nrec, MPI_Offset x)
{
    int rank, nprocs, ncid, dimid[2], varid, bad = 0;
    MPI_Offset first, cnt, r, k, start[2], count[2], numrecs = -1;
    double *b;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
    /* balanced contiguous slabs, the LAST records on rank 0 so that rank 0
     * (the numrecs writer) never holds the largest record index alone */
    {
        const int slot = nprocs - 1 - rank;
        const MPI_Offset base = nrec / nprocs, rem = nrec % nprocs;
        first = slot * base + (slot < rem ? slot : rem);
        cnt = base + (slot < rem ? 1 : 0);
    }
    b = (double *)malloc(sizeof(double) * (size_t)(nrec * x + 1));
    for (r = first; r < first + cnt; r++)
        for (k = 0; k < x; k++) b[(r - first) * x + k] = (double)r * 1000.0 + (double)k + 0.25;
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &dimid[0]));
    CHECK(ncmpi_def_dim(ncid, "x", x, &dimid[1]));
    CHECK(ncmpi_def_var(ncid, "v", NC_DOUBLE, 2, dimid, &varid));
    CHECK(ncmpi_enddef(ncid));
    start[0] = first;
    start[1] = 0;
    count[0] = cnt;
    count[1] = x;
    CHECK(ncmpi_put_vara_double_all(ncid, varid, start, count, b));
    CHECK(ncmpi_inq_dimlen(ncid, dimid[0], &numrecs));      /* MAX-synced after the collective put */
    if (numrecs != nrec) { fprintf(stderr, "rank %d numrecs %lld after put\n", rank, (long long)numrecs); nerrs++; }
    CHECK(ncmpi_close(ncid));
    CHECK(ncmpi_open(MPI_COMM_WORLD, path, NC_NOWRITE, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_inq_dimlen(ncid, 0, &numrecs));
    if (numrecs != nrec) { fprintf(stderr, "rank %d numrecs %lld on disk\n", rank, (long long)numrecs); nerrs++; }
    start[0] = 0;
    count[0] = nrec;
    CHECK(ncmpi_get_vara_double_all(ncid, 0, start, count, b));
    for (r = 0; r < nrec && !bad; r++)
        for (k = 0; k < x; k++)
            if (b[r * x + k] != (double)r * 1000.0 + (double)k + 0.25) { bad = 1; break; }
    if (bad) { fprintf(stderr, "rank %d data mismatch\n", rank); nerrs++; }
    CHECK(ncmpi_close(ncid));
    MPI_Allreduce(MPI_IN_PLACE, &nerrs, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (rank == 0) printf("{\"mode\": \"records\", \"nprocs\": %d, \"nrec\": %lld, \"errors\": %d}\n", nprocs,
                          (long long)nrec, nerrs);
    free(b);
    return nerrs != 0;
}

static int cmp_dbl(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

/* per-phase sums of libpncx (pncx_phases, include/pncx.h), looked up at run
 * time so this program links against libpnetcdf alone */
static int phases_on(void)
{
    const char *e = getenv("PNCX_PHASES");
    return e != NULL && atoi(e) != 0;
}

static void phases_reset(void)
{
    int (*on)(int) = (int (*)(int))dlsym(RTLD_DEFAULT, "pncx_phases");
    if (on) on(1);
}

/* "label": {"phase": [us per call, runs per call], ...} for phases that ran */
static void phases_print(const char *label, int calls)
{
    const char *(*name)(int) = (const char *(*)(int))dlsym(RTLD_DEFAULT, "pncx_phase_name");
    int (*rd)(int, double *, long long *) = (int (*)(int, double *, long long *))dlsym(RTLD_DEFAULT, "pncx_phase_read");
    int id, k = 0;
    if (!name || !rd || calls <= 0) return;
    printf(", \"%s\": {", label);
    for (id = 0; name(id) != NULL; id++) {
        double us = 0;
        long long n = 0;
        rd(id, &us, &n);
        if (n == 0) continue;
        printf("%s\"%s\": [%.2f, %.2f]", k++ ? ", " : "", name(id), us / calls, (double)n / calls);
    }
    printf("}");
}

/* config 1 under the reference's own access pattern (benchmarks/C/
 * pnetcdf_put_vara.c:193-209): a record variable x(time, n) NC_INT, each
 * record put exactly once with ncmpi_put_vara_int_all (appended past the
 * end of the file, numrecs written by the collective put), then each record
 * got once with ncmpi_get_vara_int_all; per-call medians, plus the put loop,
 * the get loop and the close timed whole.  Every record's values differ
 * (record r holds v + r), and every element read back is checked. */
static int mode_c1first(const char *path, MPI_Offset n, int nrec, int dev, int dbl)
{
    /* dbl: the user buffers are double (ncmpi_put/get_vara_double_all into
     * the NC_INT variable, a cross-type conversion) */
    const size_t ub = (size_t)n * (dbl ? 8 : 4);
    int *h = (int *)malloc((size_t)n * 4), *g = (int *)calloc((size_t)n, 4), ncid, dimid[2], varid, r, bad = 0;
    double *hd = dbl ? (double *)malloc(ub) : NULL, *gd = dbl ? (double *)calloc((size_t)n, 8) : NULL;
    double *tp = (double *)calloc((size_t)nrec, sizeof(double)), *tg = (double *)calloc((size_t)nrec, sizeof(double));
    double put_loop, get_loop, t_close, t0, t_open, t_create;
    void *dh = NULL, *dg = NULL;
    MPI_Offset start[2] = {0, 0}, count[2] = {1, n}, off = 0, i, nr = 0;
    double put_us[64] = {0}, first_us[64] = {0}, put_first = 0, get_first = 0;
    long long put_n[64] = {0}, first_n[64] = {0};
    for (i = 0; i < n; i++) h[i] = (int)((uint32_t)i * 2654435761u);
    if (dev) {
        dh = to_dev(NULL, ub);
        dg = to_dev(NULL, ub);
    }
    t_open = MPI_Wtime();
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    t_create = MPI_Wtime() - t_open;
    CHECK(ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &dimid[0]));
    CHECK(ncmpi_def_dim(ncid, "x", n, &dimid[1]));
    CHECK(ncmpi_def_var(ncid, "v", NC_INT, 2, dimid, &varid));
    CHECK(ncmpi_enddef(ncid));
    t_open = MPI_Wtime() - t_open;                           /* create through enddef */
    CHECK(ncmpi_inq_varoffset(ncid, varid, &off));
    if (phases_on()) phases_reset();
    put_loop = MPI_Wtime();
    for (r = 0; r < nrec; r++) {
        for (i = 0; i < n; i++) h[i] += 1;                   /* a new record's values */
        if (dbl) for (i = 0; i < n; i++) hd[i] = (double)h[i];
        if (dev && hipMemcpy(dh, dbl ? (void *)hd : (void *)h, ub, hipMemcpyHostToDevice) != hipSuccess) { fprintf(stderr, "H2D failed\n"); exit(3); }
        start[0] = r;
        if (r == 1 && phases_on()) {                         /* phases of the calls after the first */
            const char *(*name)(int) = (const char *(*)(int))dlsym(RTLD_DEFAULT, "pncx_phase_name");
            int (*rd)(int, double *, long long *) = (int (*)(int, double *, long long *))dlsym(RTLD_DEFAULT, "pncx_phase_read");
            int id;
            for (id = 0; name && rd && name(id) != NULL && id < 64; id++) rd(id, &first_us[id], &first_n[id]);
            phases_reset();
        }
        t0 = MPI_Wtime();
        if (dbl) CHECK(ncmpi_put_vara_double_all(ncid, varid, start, count, dev ? dh : (void *)hd));
        else CHECK(ncmpi_put_vara_int_all(ncid, varid, start, count, dev ? dh : (void *)h));
        tp[r] = MPI_Wtime() - t0;
    }
    put_loop = MPI_Wtime() - put_loop;
    put_first = tp[0];
    if (phases_on()) {                  /* keep the put sums for printing after the get loop */
        const char *(*name)(int) = (const char *(*)(int))dlsym(RTLD_DEFAULT, "pncx_phase_name");
        int (*rd)(int, double *, long long *) = (int (*)(int, double *, long long *))dlsym(RTLD_DEFAULT, "pncx_phase_read");
        int id;
        for (id = 0; name && rd && name(id) != NULL && id < 64; id++) rd(id, &put_us[id], &put_n[id]);
        phases_reset();
    }
    CHECK(ncmpi_inq_dimlen(ncid, dimid[0], &nr));
    if (nr != nrec) { fprintf(stderr, "c1first: numrecs %lld != %d\n", (long long)nr, nrec); nerrs++; }
    for (i = 0; i < n; i++) h[i] -= nrec;                    /* record 0's values */
    get_loop = 0;
    for (r = 0; r < nrec; r++) {
        start[0] = r;
        if (r == 1 && phases_on()) phases_reset();
        t0 = MPI_Wtime();
        if (dbl) CHECK(ncmpi_get_vara_double_all(ncid, varid, start, count, dev ? dg : (void *)gd));
        else CHECK(ncmpi_get_vara_int_all(ncid, varid, start, count, dev ? dg : (void *)g));
        tg[r] = MPI_Wtime() - t0;
        get_loop += tg[r];
        if (r == 0) get_first = tg[0];
        if (dev) from_dev(dbl ? (void *)gd : (void *)g, dg, ub);
        if (dbl) for (i = 0; i < n && !bad; i++) bad = gd[i] != (double)(int)(h[i] + r + 1);
        else for (i = 0; i < n && !bad; i++) bad = g[i] != h[i] + r + 1;
    }
    t0 = MPI_Wtime();
    CHECK(ncmpi_close(ncid));
    t_close = MPI_Wtime() - t0;
    if (bad) { fprintf(stderr, "c1first: get differs from put\n"); nerrs++; }
    qsort(tp, (size_t)nrec, sizeof(double), cmp_dbl);
    qsort(tg, (size_t)nrec, sizeof(double), cmp_dbl);
    printf("{\"mode\": \"c1first\", \"n\": %lld, \"nrec\": %d, \"dev\": %d, \"rec_offset\": %lld, "
           "\"put_ms_median\": %.5f, \"put_ms_min\": %.5f, \"get_ms_median\": %.5f, \"get_ms_min\": %.5f, "
           "\"put_loop_ms\": %.4f, \"get_loop_ms\": %.4f, \"close_ms\": %.4f, \"put_first_ms\": %.4f, "
           "\"get_first_ms\": %.4f, \"create_ms\": %.4f, \"create_to_enddef_ms\": %.4f, \"errors\": %d",
           (long long)n, nrec, dev, (long long)off, 1e3 * tp[nrec / 2], 1e3 * tp[0], 1e3 * tg[nrec / 2], 1e3 * tg[0],
           1e3 * put_loop, 1e3 * get_loop, 1e3 * t_close, 1e3 * put_first, 1e3 * get_first, 1e3 * t_create,
           1e3 * t_open, nerrs);
    if (phases_on()) {
        const char *(*name)(int) = (const char *(*)(int))dlsym(RTLD_DEFAULT, "pncx_phase_name");
        int id, k = 0;
        printf(", \"first_put_phases\": {");
        for (id = 0; name && name(id) != NULL && id < 64; id++)
            if (first_n[id] > 0)
                printf("%s\"%s\": [%.2f, %.2f]", k++ ? ", " : "", name(id), first_us[id], (double)first_n[id]);
        printf("}");
        k = 0;
        printf(", \"put_phases\": {");
        for (id = 0; name && name(id) != NULL && id < 64; id++)
            if (put_n[id] > 0)
                printf("%s\"%s\": [%.2f, %.2f]", k++ ? ", " : "", name(id), put_us[id] / (nrec - 1),
                       (double)put_n[id] / (nrec - 1));
        printf("}");
        phases_print("get_phases", nrec - 1);
    }
    printf("}\n");
    if (dev) { hipFree(dh); hipFree(dg); }
    free(h); free(g); free(hd); free(gd); free(tp); free(tg);
    return nerrs != 0;
}

/* c1first with a libpncx knob alternating between two values record by
 * record (A/B in one process, so both settings see the same box state):
 * medians of the puts and gets under each value */
static int mode_c1ab(const char *path, MPI_Offset n, int nrec, const char *knob, long long va, long long vb, int dev)
{
    int *h = (int *)malloc((size_t)n * 4), *g = (int *)calloc((size_t)n, 4), ncid, dimid[2], varid, r, bad = 0;
    void *dh = dev ? to_dev(NULL, (size_t)n * 4) : NULL, *dg = dev ? to_dev(NULL, (size_t)n * 4) : NULL;
    double *tp[2], *tg[2], t0;
    int np[2] = {0, 0}, ng[2] = {0, 0}, k;
    int (*kset)(const char *, long long) = (int (*)(const char *, long long))dlsym(RTLD_DEFAULT, "pncx_knob_set");
    MPI_Offset start[2] = {0, 0}, count[2] = {1, n}, i;
    for (k = 0; k < 2; k++) {
        tp[k] = (double *)calloc((size_t)nrec, sizeof(double));
        tg[k] = (double *)calloc((size_t)nrec, sizeof(double));
    }
    if (kset == NULL) { fprintf(stderr, "no pncx_knob_set\n"); return 1; }
    for (i = 0; i < n; i++) h[i] = (int)((uint32_t)i * 2654435761u);
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &dimid[0]));
    CHECK(ncmpi_def_dim(ncid, "x", n, &dimid[1]));
    CHECK(ncmpi_def_var(ncid, "v", NC_INT, 2, dimid, &varid));
    CHECK(ncmpi_enddef(ncid));
    for (r = 0; r < nrec; r++) {
        k = (r / 2) % 2 ^ (r % 2);                      /* A B B A A B B A ...: no order bias */
        for (i = 0; i < n; i++) h[i] += 1;
        if (dev && hipMemcpy(dh, h, (size_t)n * 4, hipMemcpyHostToDevice) != hipSuccess) { fprintf(stderr, "H2D failed\n"); exit(3); }
        start[0] = r;
        kset(knob, k ? vb : va);
        t0 = MPI_Wtime();
        CHECK(ncmpi_put_vara_int_all(ncid, varid, start, count, dev ? dh : (void *)h));
        if (r > 0) tp[k][np[k]++] = MPI_Wtime() - t0;
    }
    for (i = 0; i < n; i++) h[i] -= nrec;
    for (r = 0; r < nrec; r++) {
        k = (r / 2) % 2 ^ (r % 2);
        start[0] = r;
        kset(knob, k ? vb : va);
        t0 = MPI_Wtime();
        CHECK(ncmpi_get_vara_int_all(ncid, varid, start, count, dev ? dg : (void *)g));
        if (r > 0) tg[k][ng[k]++] = MPI_Wtime() - t0;
        if (dev) from_dev(g, dg, (size_t)n * 4);
        for (i = 0; i < n && !bad; i++) bad = g[i] != h[i] + r + 1;
    }
    kset(knob, -1);
    CHECK(ncmpi_close(ncid));
    if (bad) { fprintf(stderr, "c1ab: get differs from put\n"); nerrs++; }
    printf("{\"mode\": \"c1ab\", \"knob\": \"%s\"", knob);
    for (k = 0; k < 2; k++) {
        qsort(tp[k], (size_t)np[k], sizeof(double), cmp_dbl);
        qsort(tg[k], (size_t)ng[k], sizeof(double), cmp_dbl);
        printf(", \"%lld\": {\"put_ms\": %.4f, \"get_ms\": %.4f}", k ? vb : va, 1e3 * tp[k][np[k] / 2],
               1e3 * tg[k][ng[k] / 2]);
        free(tp[k]); free(tg[k]);
    }
    printf(", \"dev\": %d, \"errors\": %d}\n", dev, nerrs);
    if (dev) { hipFree(dh); hipFree(dg); }
    free(h); free(g);
    return nerrs != 0;
}

/* config 1 timed (bench.py's c1 leg): one open file, reps puts then reps gets.
 * With PNCX_PHASES=1 the line also carries the per-phase time of the calls
 * after the first (put_phases / get_phases, us per call). */
static int mode_c1bench(const char *path, MPI_Offset n, int reps, int dev)
{
    int *h = (int *)malloc((size_t)n * 4), *g = (int *)calloc((size_t)n, 4), ncid, dimid, varid, r, bad = 0;
    double *tp = (double *)calloc((size_t)reps, sizeof(double)), *tg = (double *)calloc((size_t)reps, sizeof(double));
    void *dh = NULL, *dg = NULL;
    MPI_Offset start[1] = {0}, count[1] = {n}, off = 0, i;
    double put_us[64] = {0};
    long long put_n[64] = {0};
    int phase_put_done = 0;
    for (i = 0; i < n; i++) h[i] = (int)((uint32_t)i * 2654435761u);
    if (dev) {
        dh = to_dev(h, (size_t)n * 4);
        dg = to_dev(NULL, (size_t)n * 4);
    }
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "x", n, &dimid));
    CHECK(ncmpi_def_var(ncid, "v", NC_INT, 1, &dimid, &varid));
    CHECK(ncmpi_enddef(ncid));
    CHECK(ncmpi_inq_varoffset(ncid, varid, &off));
    for (r = 0; r < reps; r++) {
        const double t0 = MPI_Wtime();
        if (r == 1 && phases_on()) phases_reset();
        CHECK(ncmpi_put_vara_int_all(ncid, varid, start, count, dev ? dh : (void *)h));
        tp[r] = MPI_Wtime() - t0;
    }
    if (phases_on()) phase_put_done = 1;
    if (phases_on()) {
        /* keep the put sums for printing after the get loop */
        const char *(*name)(int) = (const char *(*)(int))dlsym(RTLD_DEFAULT, "pncx_phase_name");
        int (*rd)(int, double *, long long *) = (int (*)(int, double *, long long *))dlsym(RTLD_DEFAULT, "pncx_phase_read");
        int id;
        for (id = 0; name && rd && name(id) != NULL && id < 64; id++) rd(id, &put_us[id], &put_n[id]);
    }
    for (r = 0; r < reps; r++) {
        const double t0 = MPI_Wtime();
        if (r == 1 && phases_on()) phases_reset();
        CHECK(ncmpi_get_vara_int_all(ncid, varid, start, count, dev ? dg : (void *)g));
        tg[r] = MPI_Wtime() - t0;
    }
    CHECK(ncmpi_close(ncid));
    if (dev) from_dev(g, dg, (size_t)n * 4);
    for (i = 0; i < n && !bad; i++) bad = g[i] != h[i];
    if (bad) { fprintf(stderr, "c1bench: get differs from put\n"); nerrs++; }
    qsort(tp, (size_t)reps, sizeof(double), cmp_dbl);
    qsort(tg, (size_t)reps, sizeof(double), cmp_dbl);
    printf("{\"mode\": \"c1bench\", \"n\": %lld, \"reps\": %d, \"dev\": %d, \"var_offset\": %lld, "
           "\"put_ms_median\": %.5f, \"put_ms_min\": %.5f, \"get_ms_median\": %.5f, \"get_ms_min\": %.5f, "
           "\"errors\": %d", (long long)n, reps, dev, (long long)off, 1e3 * tp[reps / 2], 1e3 * tp[0],
           1e3 * tg[reps / 2], 1e3 * tg[0], nerrs);
    if (phase_put_done && reps > 1) {
        const char *(*name)(int) = (const char *(*)(int))dlsym(RTLD_DEFAULT, "pncx_phase_name");
        int id, k = 0;
        printf(", \"put_phases\": {");
        for (id = 0; name && name(id) != NULL && id < 64; id++)
            if (put_n[id] > 0)
                printf("%s\"%s\": [%.2f, %.2f]", k++ ? ", " : "", name(id), put_us[id] / (reps - 1),
                       (double)put_n[id] / (reps - 1));
        printf("}");
        phases_print("get_phases", reps - 1);
    }
    printf("}\n");
    if (dev) { hipFree(dh); hipFree(dg); }
    free(h); free(g); free(tp); free(tg);
    return nerrs != 0;
}

/* numrecs as the FILE holds it (big-endian at byte 4; 8 bytes for CDF-5) */
static long long file_numrecs(const char *path)
{
    unsigned char b[8];
    long long v = 0;
    int i;
    FILE *f = fopen(path, "rb");
    if (f == NULL || fseek(f, 4, SEEK_SET) != 0 || fread(b, 1, 8, f) != 8) { if (f) fclose(f); return -1; }
    fclose(f);
    for (i = 0; i < 8; i++) v = (v << 8) | b[i];
    return v;
}

static int mode_numrecs(const char *path)
{
    int rank, nprocs, ncid, dimid[2], vr, vf, k;
    long long seen[3];
    int buf[16];
    MPI_Offset start[2], count[2];
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
    for (k = 0; k < 16; k++) buf[k] = rank * 100 + k;
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &dimid[0]));
    CHECK(ncmpi_def_dim(ncid, "x", 16, &dimid[1]));
    CHECK(ncmpi_def_var(ncid, "r", NC_INT, 2, dimid, &vr));
    CHECK(ncmpi_def_var(ncid, "f", NC_INT, 1, &dimid[1], &vf));
    CHECK(ncmpi_enddef(ncid));
    /* put 1: rank r writes record r */
    start[0] = rank; start[1] = 0; count[0] = 1; count[1] = 16;
    CHECK(ncmpi_put_vara_int_all(ncid, vr, start, count, buf));
    MPI_Barrier(MPI_COMM_WORLD);
    seen[0] = file_numrecs(path);
    /* a fixed-size variable: numrecs unchanged */
    start[0] = 0; count[0] = 16;
    CHECK(ncmpi_put_vara_int_all(ncid, vf, start, count, buf));
    MPI_Barrier(MPI_COMM_WORLD);
    seen[1] = file_numrecs(path);
    /* put 2: only rank 0 writes, record nprocs + 1 (others zero-length) */
    start[0] = nprocs + 1; start[1] = 0; count[0] = rank == 0 ? 1 : 0; count[1] = 16;
    CHECK(ncmpi_put_vara_int_all(ncid, vr, start, count, buf));
    MPI_Barrier(MPI_COMM_WORLD);
    seen[2] = file_numrecs(path);
    CHECK(ncmpi_close(ncid));
    MPI_Allreduce(MPI_IN_PLACE, &nerrs, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (rank == 0)
        printf("{\"mode\": \"numrecs\", \"nprocs\": %d, \"after_rec_put\": %lld, \"after_fix_put\": %lld, "
               "\"after_second_rec_put\": %lld, \"at_close\": %lld, \"errors\": %d}\n", nprocs, seen[0], seen[1],
               seen[2], file_numrecs(path), nerrs);
    return nerrs != 0;
}

static int mode_openfail(const char *dir)
{
    char a[512], b[512], c[512];
    int rank, nprocs, ncid, dimid, varid, id2 = -7, e_open, e_create, got[8], i, vals[8];
    MPI_Offset start[1] = {0}, count[1] = {8};
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
    for (i = 0; i < 8; i++) vals[i] = 10 * rank + i;
    snprintf(a, sizeof a, "%s/a.nc", dir);
    snprintf(c, sizeof c, "%s/c.nc", dir);
    /* the last rank names a file that does not exist / a directory that does not */
    if (rank == nprocs - 1) snprintf(b, sizeof b, "%s/missing.nc", dir);
    else snprintf(b, sizeof b, "%s/a.nc", dir);
    CHECK(ncmpi_create(MPI_COMM_WORLD, a, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "x", 8 * nprocs, &dimid));
    CHECK(ncmpi_def_var(ncid, "v", NC_INT, 1, &dimid, &varid));
    CHECK(ncmpi_enddef(ncid));
    e_open = ncmpi_open(MPI_COMM_WORLD, b, NC_NOWRITE, MPI_INFO_NULL, &id2);
    if (rank == nprocs - 1) snprintf(c, sizeof c, "%s/nodir/c.nc", dir);
    e_create = ncmpi_create(MPI_COMM_WORLD, c, NC_CLOBBER, MPI_INFO_NULL, &id2);
    /* the first file is still open and usable on every rank */
    start[0] = 8 * rank;
    CHECK(ncmpi_put_vara_int_all(ncid, varid, start, count, vals));
    CHECK(ncmpi_get_vara_int_all(ncid, varid, start, count, got));
    for (i = 0; i < 8; i++)
        if (got[i] != vals[i]) { fprintf(stderr, "rank %d: a.nc data lost\n", rank); nerrs++; break; }
    CHECK(ncmpi_close(ncid));
    MPI_Allreduce(MPI_IN_PLACE, &nerrs, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (rank == 0) {
        FILE *f;
        snprintf(c, sizeof c, "%s/c.nc", dir);
        f = fopen(c, "rb");
        printf("{\"mode\": \"openfail\", \"nprocs\": %d, \"open\": %d, \"create\": %d, \"c_exists\": %d, "
               "\"errors\": %d}\n", nprocs, e_open, e_create, f != NULL, nerrs);
        if (f) fclose(f);
    }
    return nerrs != 0;
}

static int mode_bputshort(const char *path)
{
    int ncid, dimid, varid, req = -5, vals[16] = {0}, e_short, e_ok, st = -1;
    MPI_Offset start[1] = {0}, count[1] = {16};
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "x", 16, &dimid));
    CHECK(ncmpi_def_var(ncid, "v", NC_INT, 1, &dimid, &varid));
    CHECK(ncmpi_enddef(ncid));
    CHECK(ncmpi_buffer_attach(ncid, 1024));
    e_short = ncmpi_bput_vara(ncid, varid, start, count, vals, 8, MPI_INT, &req);
    e_ok = ncmpi_bput_vara(ncid, varid, start, count, vals, 16, MPI_INT, &req);
    CHECK(ncmpi_wait_all(ncid, 1, &req, &st));
    CHECK(ncmpi_buffer_detach(ncid));
    CHECK(ncmpi_close(ncid));
    printf("{\"mode\": \"bputshort\", \"short\": %d, \"exact\": %d, \"status\": %d, \"errors\": %d}\n", e_short, e_ok,
           st, nerrs);
    return nerrs != 0;
}

/* Derived buftypes over hipMalloc'ed (dev = 1) or host (dev = 0) buffers
 * through the flexible varn and bput calls (ncmpio_i_varn.m4:165-231,
 * ncmpio_i_getput.m4:266-310): the user buffer is a 10 x 14 int array whose
 * 8 x 12 interior (one ghost cell around) is an MPI subarray type.
 *   a NC_INT:    ncmpi_put_varn_all, two boxes of 4 rows
 *   b NC_SHORT:  ncmpi_bput_vara (values out of short range: NC_ERANGE at post)
 *   c NC_DOUBLE: ncmpi_iput_varn + wait_all
 * then ncmpi_get_varn_all of a and ncmpi_iget_varn of c into fresh
 * subarray buffers whose ghost cells must survive.  Values: v[i] =
 * (i * 7919) % 80000 - 40000 over the interior in row-major order. */
static int mode_flexdev(const char *path, int dev)
{
    enum { Y = 8, X = 12, GY = 10, GX = 14 };
    int ncid, dims[2], va, vb, vc, req[2] = {-1, -1}, st[2] = {-9, -9}, e_bput, i, y, x, bad = 0;
    int *h = (int *)calloc(GY * GX, sizeof(int)), *g1 = (int *)malloc(GY * GX * sizeof(int)),
        *g2 = (int *)malloc(GY * GX * sizeof(int));
    void *buf, *d1 = NULL, *d2 = NULL;
    MPI_Datatype sub;
    int sizes[2] = {GY, GX}, subs[2] = {Y, X}, starts[2] = {1, 1};
    MPI_Offset s0[2] = {0, 0}, s1[2] = {4, 0}, c4[2] = {4, X}, c8[2] = {Y, X};
    MPI_Offset *vs[2] = {s0, s1}, *vc4[2] = {c4, c4};
    for (i = 0; i < GY * GX; i++) h[i] = -1;
    for (y = 0; y < Y; y++)
        for (x = 0; x < X; x++) h[(y + 1) * GX + x + 1] = (int)(((long long)(y * X + x) * 7919) % 80000) - 40000;
    MPI_Type_create_subarray(2, sizes, subs, starts, MPI_ORDER_C, MPI_INT, &sub);
    MPI_Type_commit(&sub);
    buf = dev ? to_dev(h, GY * GX * sizeof(int)) : (void *)h;
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_def_dim(ncid, "y", Y, &dims[0]));
    CHECK(ncmpi_def_dim(ncid, "x", X, &dims[1]));
    CHECK(ncmpi_def_var(ncid, "a", NC_INT, 2, dims, &va));
    CHECK(ncmpi_def_var(ncid, "b", NC_SHORT, 2, dims, &vb));
    CHECK(ncmpi_def_var(ncid, "c", NC_DOUBLE, 2, dims, &vc));
    CHECK(ncmpi_enddef(ncid));
    CHECK(ncmpi_buffer_attach(ncid, Y * X * 8));
    CHECK(ncmpi_put_varn_all(ncid, va, 2, vs, vc4, buf, 1, sub));
    e_bput = ncmpi_bput_vara(ncid, vb, s0, c8, buf, 1, sub, &req[0]);
    CHECK(ncmpi_iput_varn(ncid, vc, 2, vs, vc4, buf, 1, sub, &req[1]));
    CHECK(ncmpi_wait_all(ncid, 2, req, st));
    CHECK(ncmpi_buffer_detach(ncid));
    /* reads back into subarray buffers whose ghosts hold -5 / -6 */
    for (i = 0; i < GY * GX; i++) { g1[i] = -5; g2[i] = -6; }
    if (dev) { d1 = to_dev(g1, GY * GX * sizeof(int)); d2 = to_dev(g2, GY * GX * sizeof(int)); }
    CHECK(ncmpi_get_varn_all(ncid, va, 2, vs, vc4, dev ? d1 : (void *)g1, 1, sub));
    CHECK(ncmpi_iget_varn(ncid, vc, 2, vs, vc4, dev ? d2 : (void *)g2, 1, sub, &req[0]));
    CHECK(ncmpi_wait_all(ncid, 1, req, NULL));
    CHECK(ncmpi_close(ncid));
    if (dev) {
        from_dev(g1, d1, GY * GX * sizeof(int));
        from_dev(g2, d2, GY * GX * sizeof(int));
        hipFree(d1);
        hipFree(d2);
        hipFree(buf);
    }
    for (y = 0; y < GY && !bad; y++)
        for (x = 0; x < GX && !bad; x++) {
            const int in = y >= 1 && y <= Y && x >= 1 && x <= X, k = y * GX + x;
            if (g1[k] != (in ? h[k] : -5) || g2[k] != (in ? h[k] : -6)) {
                fprintf(stderr, "flexdev: get mismatch at (%d, %d): %d %d\n", y, x, g1[k], g2[k]);
                bad = 1;
            }
        }
    nerrs += bad;
    MPI_Type_free(&sub);
    printf("{\"mode\": \"flexdev\", \"dev\": %d, \"bput\": %d, \"wait_status\": [%d, %d], \"errors\": %d}\n",
           dev, e_bput, st[0], st[1], nerrs);
    free(h); free(g1); free(g2);
    return nerrs != 0;
}

/* errors the dispatcher returns before any conversion (var_getput.m4
 * sanity_check / check_start_count_stride, file.c, attr_getput.m4) */
static int mode_errors(const char *dir)
{
    char path[512];
    int ncid, dimid[2], v, vt, vr, e, i4[4] = {0}, req;
    MPI_Offset st[2] = {0, 0}, ct[2] = {1, 1}, big[2] = {5, 0}, neg[2] = {-1, 1}, st1[2] = {1, 0}, sd0[2] = {0, 0};
    float f = 1.0f;
    snprintf(path, sizeof path, "%s/errors.nc", dir);
#define R(name, call) printf("%s %d\n", name, (call))
    R("create_bad_path", ncmpi_create(MPI_COMM_WORLD, "", NC_CLOBBER, MPI_INFO_NULL, &ncid));
    R("create_both_formats", ncmpi_create(MPI_COMM_WORLD, path, NC_64BIT_DATA | NC_64BIT_OFFSET, MPI_INFO_NULL, &ncid));
    R("create_netcdf4", ncmpi_create(MPI_COMM_WORLD, path, NC_NETCDF4, MPI_INFO_NULL, &ncid));
    e = ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER, MPI_INFO_NULL, &ncid);
    R("create", e);
    R("noclobber_exists", ncmpi_create(MPI_COMM_WORLD, path, NC_NOCLOBBER, MPI_INFO_NULL, &v));
    R("def_dim", ncmpi_def_dim(ncid, "t", NC_UNLIMITED, &dimid[0]));
    R("def_dim_x", ncmpi_def_dim(ncid, "x", 4, &dimid[1]));
    R("def_dim_second_unlimited", ncmpi_def_dim(ncid, "u2", NC_UNLIMITED, &v));
    R("def_dim_name_in_use", ncmpi_def_dim(ncid, "x", 4, &v));
    R("def_var_cdf1_int64", ncmpi_def_var(ncid, "w", NC_INT64, 1, &dimid[1], &v));
    R("def_var_badtype", ncmpi_def_var(ncid, "w", 99, 1, &dimid[1], &v));
    R("def_var", ncmpi_def_var(ncid, "v", NC_INT, 1, &dimid[1], &v));
    R("def_var_text", ncmpi_def_var(ncid, "c", NC_CHAR, 1, &dimid[1], &vt));
    R("def_var_rec", ncmpi_def_var(ncid, "r", NC_FLOAT, 2, dimid, &vr));
    R("put_in_define_mode", ncmpi_put_vara_int_all(ncid, v, st, ct, i4));
    R("inq_bad_ncid", ncmpi_inq(12345, NULL, NULL, NULL, NULL));
    R("put_att_echar", ncmpi_put_att_int(ncid, NC_GLOBAL, "a", NC_CHAR, 1, i4));
    R("put_att_strict_cdf2", ncmpi_put_att_int(ncid, NC_GLOBAL, "a", NC_UINT, 1, i4));
    R("put_att_negative_len", ncmpi_put_att_text(ncid, NC_GLOBAL, "a", -1, "x"));
    R("put_att_text", ncmpi_put_att_text(ncid, NC_GLOBAL, "title", 5, "hello"));
    R("inq_att_missing", ncmpi_inq_att(ncid, NC_GLOBAL, "nope", NULL, NULL));
    R("enddef", ncmpi_enddef(ncid));
    R("enddef_again", ncmpi_enddef(ncid));
    R("def_dim_in_data_mode", ncmpi_def_dim(ncid, "y", 4, &v));
    R("put_global", ncmpi_put_vara_int_all(ncid, NC_GLOBAL, st, ct, i4));
    R("put_bad_varid", ncmpi_put_vara_int_all(ncid, 77, st, ct, i4));
    R("put_indep_in_coll_mode", ncmpi_put_vara_int(ncid, 0, st, ct, i4));
    R("put_text_into_int", ncmpi_put_vara_text_all(ncid, 0, st, ct, "a"));
    R("put_int_into_text", ncmpi_put_vara_int_all(ncid, vt, st, ct, i4));
    R("put_start_out_of_bound", ncmpi_put_vara_int_all(ncid, 0, big, ct, i4));
    R("put_start_negative", ncmpi_put_vara_int_all(ncid, 0, neg, ct, i4));
    R("put_edge", ncmpi_put_vara_int_all(ncid, 0, st1, big, i4));
    R("put_stride_zero", ncmpi_put_vars_int_all(ncid, 0, st, ct, sd0, i4));
    R("get_rec_beyond_numrecs", ncmpi_get_vara_float_all(ncid, vr, st, ct, &f));
    R("put_vara_null_count", ncmpi_put_vara_int_all(ncid, 0, st, NULL, i4));
    R("flex_ignore_derived", ncmpi_put_vara_all(ncid, 0, st, ct, i4, NC_COUNT_IGNORE, MPI_2INT));
    R("bput_no_buffer", ncmpi_bput_vara_int(ncid, 0, st, ct, i4, &req));
    R("wait_indep_in_coll_mode", ncmpi_wait(ncid, NC_REQ_ALL, NULL, NULL));
    R("begin_indep", ncmpi_begin_indep_data(ncid));
    R("put_coll_in_indep_mode", ncmpi_put_vara_int_all(ncid, 0, st, ct, i4));
    R("wait_all_in_indep_mode", ncmpi_wait_all(ncid, NC_REQ_ALL, NULL, NULL));
    R("end_indep", ncmpi_end_indep_data(ncid));
    R("redef", ncmpi_redef(ncid));
    R("redef_again", ncmpi_redef(ncid));
    R("del_att", ncmpi_del_att(ncid, NC_GLOBAL, "title"));
    R("enddef2", ncmpi_enddef(ncid));
    R("del_att_data_mode", ncmpi_del_att(ncid, NC_GLOBAL, "title"));
    R("vard_deprecated", ncmpi_put_vard_all(ncid, 0, MPI_INT, i4, 1, MPI_INT));
    R("malloc_size_disabled", ncmpi_inq_malloc_size(&st[0]));
    R("close", ncmpi_close(ncid));
    R("close_again", ncmpi_close(ncid));
    R("open_missing", ncmpi_open(MPI_COMM_WORLD, "/nonexistent/x.nc", NC_NOWRITE, MPI_INFO_NULL, &ncid));
    e = ncmpi_open(MPI_COMM_WORLD, path, NC_NOWRITE, MPI_INFO_NULL, &ncid);
    R("open_ro", e);
    R("put_read_only", ncmpi_put_vara_int_all(ncid, 0, st, ct, i4));
    R("redef_read_only", ncmpi_redef(ncid));
    {
        int nd = -1, nv = -1, na = -1, ul = -2, fmt = -1;
        MPI_Offset len = -1;
        char name[NC_MAX_NAME + 1];
        R("inq", ncmpi_inq(ncid, &nd, &nv, &na, &ul));
        printf("inq_values %d %d %d %d\n", nd, nv, na, ul);
        R("inq_format", ncmpi_inq_format(ncid, &fmt));
        printf("format %d\n", fmt);
        R("inq_dim", ncmpi_inq_dim(ncid, 1, name, &len));
        printf("dim1 %s %lld\n", name, (long long)len);
        R("inq_varname", ncmpi_inq_varname(ncid, 2, name));
        printf("var2 %s\n", name);
        R("inq_attlen", ncmpi_inq_attlen(ncid, NC_GLOBAL, "title", &len));
        R("inq_num_rec_vars", ncmpi_inq_num_rec_vars(ncid, &nv));
        printf("num_rec_vars %d\n", nv);
    }
    R("close_ro", ncmpi_close(ncid));
#undef R
    return 0;
}

static int mode_header(const char *path)
{
    int ncid, d[3], v[4];
    CHECK(ncmpi_create(MPI_COMM_WORLD, path, NC_CLOBBER | NC_64BIT_OFFSET, MPI_INFO_NULL, &ncid));
    CHECK(ncmpi_put_att_text(ncid, NC_GLOBAL, "title", 14, "shared header"));
    CHECK(ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &d[0]));
    CHECK(ncmpi_def_dim(ncid, "lat", 90, &d[1]));
    CHECK(ncmpi_def_dim(ncid, "lon", 180, &d[2]));
    CHECK(ncmpi_def_var(ncid, "temp", NC_FLOAT, 3, d, &v[0]));
    CHECK(ncmpi_def_var(ncid, "lat", NC_DOUBLE, 1, &d[1], &v[1]));
    CHECK(ncmpi_def_var(ncid, "flag", NC_BYTE, 2, &d[1], &v[2]));
    CHECK(ncmpi_def_var(ncid, "name", NC_CHAR, 1, &d[2], &v[3]));
    CHECK(ncmpi_put_att_text(ncid, v[0], "units", 1, "K"));
    CHECK(ncmpi_enddef(ncid));
    CHECK(ncmpi_redef(ncid));
    CHECK(ncmpi_put_att_text(ncid, NC_GLOBAL, "history", 7, "redef'd"));
    CHECK(ncmpi_enddef(ncid));
    CHECK(ncmpi_close(ncid));
    MPI_Allreduce(MPI_IN_PLACE, &nerrs, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    return nerrs != 0;
}

/* ------------------------------------------------------------------ pthread */
typedef struct {
    const char *prefix;
    int id, nthreads, coll, dev;
    MPI_Offset nx, ny;
    pthread_barrier_t *barr;
    char out[512];
    int errs;
} pt_arg;

#define TCHECK(call)                                                                                      \
    do {                                                                                                  \
        int _e = (call);                                                                                  \
        if (_e != NC_NOERR) {                                                                             \
            fprintf(stderr, "thread %d %s:%d: %s -> %d %s\n", a->id, __FILE__, __LINE__, #call, _e,          \
                    ncmpi_strerror(_e));                                                                  \
            a->errs++;                                                                                    \
        }                                                                                                 \
    } while (0)

static int pt_ival(int id, int r, MPI_Offset i) { return (int)((uint32_t)id * 1000003u + (uint32_t)r * 7919u + (uint32_t)i); }
static double pt_dval(int id, MPI_Offset i) { return (double)id + 0.5 * (double)i; }

static void *pt_main(void *p)
{
    pt_arg *a = (pt_arg *)p;
    const MPI_Offset nx = a->nx, ny = a->ny;
    int *ib = (int *)malloc(sizeof(int) * (size_t)nx);
    double *db = (double *)malloc(sizeof(double) * (size_t)(nx * ny));
    void *dib = NULL, *ddb = NULL;
    char fn[1024];
    int ncid, dimid[2], varid[2], r, id = a->id;
    MPI_Offset start[2], count[2], i, ioff = -1, doff = -1, recsize = -1;
    MPI_Info info;
    snprintf(fn, sizeof fn, "%s.%d", a->prefix, id);
    MPI_Info_create(&info);
    MPI_Info_set(info, "nc_var_align_size", "1");
    TCHECK(ncmpi_create(MPI_COMM_SELF, fn, NC_CLOBBER, info, &ncid));
    MPI_Info_free(&info);
    TCHECK(ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &dimid[0]));
    TCHECK(ncmpi_def_dim(ncid, "X", nx, &dimid[1]));
    TCHECK(ncmpi_def_var(ncid, "ivar", NC_INT, 2, dimid, &varid[0]));
    TCHECK(ncmpi_def_dim(ncid, "Y", ny, &dimid[0]));
    TCHECK(ncmpi_def_var(ncid, "dvar", NC_DOUBLE, 2, dimid, &varid[1]));
    TCHECK(ncmpi_enddef(ncid));
    if (!a->coll) TCHECK(ncmpi_begin_indep_data(ncid));
    if (a->dev) { dib = to_dev(NULL, sizeof(int) * (size_t)nx); ddb = to_dev(NULL, sizeof(double) * (size_t)(nx * ny)); }
    for (r = 0; r <= 2; r += 2) {                         /* records 0 and 2 (tst_pthread.c:186-207) */
        for (i = 0; i < nx; i++) ib[i] = pt_ival(id, r, i);
        if (a->dev && hipMemcpy(dib, ib, sizeof(int) * (size_t)nx, hipMemcpyHostToDevice) != hipSuccess) a->errs++;
        start[0] = r; start[1] = 0; count[0] = 1; count[1] = nx;
        if (a->coll) TCHECK(ncmpi_put_vara_int_all(ncid, varid[0], start, count, a->dev ? dib : (void *)ib));
        else TCHECK(ncmpi_put_vara_int(ncid, varid[0], start, count, a->dev ? dib : (void *)ib));
    }
    for (i = 0; i < nx * ny; i++) db[i] = pt_dval(id, i);
    if (a->dev && hipMemcpy(ddb, db, sizeof(double) * (size_t)(nx * ny), hipMemcpyHostToDevice) != hipSuccess) a->errs++;
    if (a->coll) TCHECK(ncmpi_put_var_double_all(ncid, varid[1], a->dev ? ddb : (void *)db));
    else TCHECK(ncmpi_put_var_double(ncid, varid[1], a->dev ? ddb : (void *)db));
    TCHECK(ncmpi_sync(ncid));
    TCHECK(ncmpi_inq_varoffset(ncid, varid[0], &ioff));
    TCHECK(ncmpi_inq_varoffset(ncid, varid[1], &doff));
    TCHECK(ncmpi_inq_recsize(ncid, &recsize));
    TCHECK(ncmpi_close(ncid));
    pthread_barrier_wait(a->barr);                        /* every file is written (tst_pthread.c:226) */
    id = (id + 1) % a->nthreads;                          /* another thread's file (:232-234) */
    snprintf(fn, sizeof fn, "%s.%d", a->prefix, id);
    TCHECK(ncmpi_open(MPI_COMM_SELF, fn, NC_NOWRITE, MPI_INFO_NULL, &ncid));
    if (!a->coll) TCHECK(ncmpi_begin_indep_data(ncid));
    TCHECK(ncmpi_inq_varid(ncid, "ivar", &varid[0]));
    TCHECK(ncmpi_inq_varid(ncid, "dvar", &varid[1]));
    for (r = 0; r <= 2; r += 2) {
        for (i = 0; i < nx; i++) ib[i] = -1;
        if (a->dev) (void)hipMemset(dib, 0xff, sizeof(int) * (size_t)nx);
        start[0] = r; start[1] = 0; count[0] = 1; count[1] = nx;
        if (a->coll) TCHECK(ncmpi_get_vara_int_all(ncid, varid[0], start, count, a->dev ? dib : (void *)ib));
        else TCHECK(ncmpi_get_vara_int(ncid, varid[0], start, count, a->dev ? dib : (void *)ib));
        if (a->dev) from_dev(ib, dib, sizeof(int) * (size_t)nx);
        for (i = 0; i < nx; i++)
            if (ib[i] != pt_ival(id, r, i)) {
                fprintf(stderr, "thread %d: file %d record %d element %lld: %d != %d\n", a->id, id, r, (long long)i,
                        ib[i], pt_ival(id, r, i));
                a->errs++;
                break;
            }
    }
    for (i = 0; i < nx * ny; i++) db[i] = -1.0;
    if (a->dev) (void)hipMemset(ddb, 0xff, sizeof(double) * (size_t)(nx * ny));
    if (a->coll) TCHECK(ncmpi_get_var_double_all(ncid, varid[1], a->dev ? ddb : (void *)db));
    else TCHECK(ncmpi_get_var_double(ncid, varid[1], a->dev ? ddb : (void *)db));
    if (a->dev) from_dev(db, ddb, sizeof(double) * (size_t)(nx * ny));
    for (i = 0; i < nx * ny; i++)
        if (db[i] != pt_dval(id, i)) {
            fprintf(stderr, "thread %d: file %d dvar element %lld: %g != %g\n", a->id, id, (long long)i, db[i],
                    pt_dval(id, i));
            a->errs++;
            break;
        }
    TCHECK(ncmpi_close(ncid));
    if (a->dev) { hipFree(dib); hipFree(ddb); }
    free(ib);
    free(db);
    snprintf(a->out, sizeof a->out,
             "{\"mode\": \"pthread\", \"thread\": %d, \"file\": \"%s.%d\", \"ivar_off\": %lld, \"dvar_off\": %lld, "
             "\"recsize\": %lld, \"errors\": %d}", a->id, a->prefix, a->id, (long long)ioff, (long long)doff,
             (long long)recsize, a->errs);
    return NULL;
}

/* define-mode traffic from many threads at once (no data call, so no GPU
 * needed): each thread creates, defines, ends define mode, closes, reopens,
 * looks its variable up and closes its own file, iters times; the ncid
 * table (pnc_dispatch.c) hands out and retires ids under its mutex.  At the
 * end no file may be left open. */
typedef struct { const char *prefix; int id, iters, errs; } ph_arg;

static void *ph_main(void *p)
{
    ph_arg *a = (ph_arg *)p;
    char fn[1024];
    int k;
    snprintf(fn, sizeof fn, "%s.%d", a->prefix, a->id);
    for (k = 0; k < a->iters; k++) {
        int ncid = -1, ncid2 = -1, d[2], v, v2 = -1, e;
        MPI_Offset len = -1;
        e = ncmpi_create(MPI_COMM_SELF, fn, NC_CLOBBER | NC_64BIT_DATA, MPI_INFO_NULL, &ncid);
        if (!e) e = ncmpi_def_dim(ncid, "time", NC_UNLIMITED, &d[0]);
        if (!e) e = ncmpi_def_dim(ncid, "x", 16 + a->id, &d[1]);
        if (!e) e = ncmpi_def_var(ncid, "v", NC_INT, 2, d, &v);
        if (!e) e = ncmpi_enddef(ncid);
        if (!e) e = ncmpi_close(ncid);
        if (!e) e = ncmpi_open(MPI_COMM_SELF, fn, NC_NOWRITE, MPI_INFO_NULL, &ncid2);
        if (!e) e = ncmpi_inq_varid(ncid2, "v", &v2);
        if (!e) e = ncmpi_inq_dimlen(ncid2, 1, &len);
        if (!e && (v2 != v || len != 16 + a->id)) e = NC_EINTERNAL;
        if (!e) e = ncmpi_close(ncid2);
        if (e) {
            fprintf(stderr, "thread %d iteration %d: %d %s\n", a->id, k, e, ncmpi_strerror(e));
            a->errs++;
            break;
        }
    }
    return NULL;
}

static int mode_pthread_hdr(const char *prefix, int nthreads, int iters, int provided)
{
    ph_arg *args = (ph_arg *)calloc((size_t)nthreads, sizeof(ph_arg));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    int t, errs = 0, nopen = -1;
    if (provided < MPI_THREAD_MULTIPLE) {
        fprintf(stderr, "MPI_Init_thread gave thread level %d < MPI_THREAD_MULTIPLE\n", provided);
        return 1;
    }
    for (t = 0; t < nthreads; t++) {
        args[t].prefix = prefix; args[t].id = t; args[t].iters = iters;
        if (pthread_create(&th[t], NULL, ph_main, &args[t]) != 0) { fprintf(stderr, "pthread_create\n"); return 1; }
    }
    for (t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        errs += args[t].errs;
    }
    CHECK(ncmpi_inq_files_opened(&nopen, NULL));
    printf("{\"mode\": \"pthreadhdr\", \"threads\": %d, \"iters\": %d, \"files_open\": %d, \"errors\": %d}\n",
           nthreads, iters, nopen, errs + nerrs);
    free(args);
    free(th);
    return errs + nerrs != 0 || nopen != 0;
}

static int mode_pthread(const char *prefix, int nthreads, MPI_Offset nx, MPI_Offset ny, int coll, int dev, int provided)
{
    pt_arg *args = (pt_arg *)calloc((size_t)nthreads, sizeof(pt_arg));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    pthread_barrier_t barr;
    int t, errs = 0, ncid;
    if (provided < MPI_THREAD_MULTIPLE) {
        fprintf(stderr, "MPI_Init_thread gave thread level %d < MPI_THREAD_MULTIPLE\n", provided);
        return 1;
    }
    pthread_barrier_init(&barr, NULL, (unsigned)nthreads);
    for (t = 0; t < nthreads; t++) {
        args[t].prefix = prefix; args[t].id = t; args[t].nthreads = nthreads; args[t].coll = coll;
        args[t].dev = dev; args[t].nx = nx; args[t].ny = ny; args[t].barr = &barr;
        if (pthread_create(&th[t], NULL, pt_main, &args[t]) != 0) { fprintf(stderr, "pthread_create\n"); return 1; }
    }
    for (t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        errs += args[t].errs;
        printf("%s\n", args[t].out);
    }
    pthread_barrier_destroy(&barr);
    for (t = 0; t < nthreads; t++) {                      /* every file opens again (tst_pthread.c:349-358) */
        char fn[1024];
        snprintf(fn, sizeof fn, "%s.%d", prefix, t);
        CHECK(ncmpi_open(MPI_COMM_SELF, fn, NC_NOWRITE, MPI_INFO_NULL, &ncid));
        CHECK(ncmpi_close(ncid));
    }
    printf("{\"mode\": \"pthread\", \"threads\": %d, \"errors\": %d}\n", nthreads, errs + nerrs);
    free(args);
    free(th);
    return errs + nerrs != 0;
}

int main(int argc, char **argv)
{
    int rc = 2, provided = 0;
    if (argc >= 2 && strncmp(argv[1], "pthread", 7) == 0) MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
    else MPI_Init(&argc, &argv);
    if (argc >= 5 && strcmp(argv[1], "c1") == 0)
        rc = mode_c1(argv[2], argv[3], atoll(argv[4]), argc >= 6 ? atoi(argv[5]) : 0);
    else if (argc >= 6 && strcmp(argv[1], "c1bench") == 0)
        rc = mode_c1bench(argv[2], atoll(argv[3]), atoi(argv[4]), atoi(argv[5]));
    else if (argc >= 6 && strcmp(argv[1], "c1first") == 0)
        rc = mode_c1first(argv[2], atoll(argv[3]), atoi(argv[4]), atoi(argv[5]),
                          argc >= 7 && strcmp(argv[6], "double") == 0);
    else if (argc >= 8 && strcmp(argv[1], "c1ab") == 0)
        rc = mode_c1ab(argv[2], atoll(argv[3]), atoi(argv[4]), argv[5], atoll(argv[6]), atoll(argv[7]),
                       argc >= 9 ? atoi(argv[8]) : 0);
    else if (argc >= 3 && strcmp(argv[1], "numrecs") == 0) rc = mode_numrecs(argv[2]);
    else if (argc >= 3 && strcmp(argv[1], "openfail") == 0) rc = mode_openfail(argv[2]);
    else if (argc >= 3 && strcmp(argv[1], "bputshort") == 0) rc = mode_bputshort(argv[2]);
    else if (argc >= 7 && strcmp(argv[1], "putvara") == 0)
        rc = mode_putvara(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]),
                          argc >= 8 ? atoi(argv[7]) : 0);
    else if (argc >= 7 && strcmp(argv[1], "c4") == 0)
        rc = mode_c4(argv[2], argv[3], argv[4], atoll(argv[5]), atoi(argv[6]), argc >= 8 ? atoi(argv[7]) : 0);
    else if (argc >= 5 && strcmp(argv[1], "records") == 0) rc = mode_records(argv[2], atoll(argv[3]), atoll(argv[4]));
    else if (argc >= 3 && strcmp(argv[1], "errors") == 0) rc = mode_errors(argv[2]);
    else if (argc >= 3 && strcmp(argv[1], "header") == 0) rc = mode_header(argv[2]);
    else if (argc >= 4 && strcmp(argv[1], "flexdev") == 0) rc = mode_flexdev(argv[2], atoi(argv[3]));
    else if (argc >= 5 && strcmp(argv[1], "pthreadhdr") == 0)
        rc = mode_pthread_hdr(argv[2], atoi(argv[3]), atoi(argv[4]), provided);
    else if (argc >= 7 && strcmp(argv[1], "pthread") == 0)
        rc = mode_pthread(argv[2], atoi(argv[3]), atoll(argv[4]), atoll(argv[5]), atoi(argv[6]),
                          argc >= 8 ? atoi(argv[7]) : 0, provided);
    else fprintf(stderr, "usage: see the header of api_check.c\n");
    MPI_Finalize();
    return rc;
}
