/*
 * flex_check.c -- parity checks of the flexible API (MPI derived buftypes)
 * against MPI itself.  Test infrastructure, built by tests/mpi/Makefile.
 *
 *   flex_check flatten       (CPU) pncx_mpi_type_flatten of each datatype in
 *                            the suite, replayed as a host pack, must equal
 *                            MPI_Pack of the same buffer byte for byte; the
 *                            error cases must return the reference's codes.
 *   flex_check file <dir>    (GPU) for each datatype x conversion: a put
 *                            through pncx_ncmpi_put_varm with the derived
 *                            type must write the same file bytes as
 *                            MPI_Pack + a contiguous put (the reference's
 *                            order of work, ncmpio_util.c:620-652, 716-765);
 *                            a get must equal a contiguous get + MPI_Unpack
 *                            (bytes between the runs untouched); same for
 *                            iput/iget + wait_all.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pncx_mpi.h"

#define NT 16
typedef struct tcase {
    const char *name;
    MPI_Datatype t;
    int bufcount;
} tcase;

static int ntc = 0;
static tcase tc[NT];

static void add(const char *name, MPI_Datatype t, int bufcount)
{
    MPI_Type_commit(&t);
    tc[ntc].name = name;
    tc[ntc].t = t;
    tc[ntc].bufcount = bufcount;
    ntc++;
}

/* the datatype suite; every type is built from `e` only */
static void build_suite(MPI_Datatype e, int es)
{
    MPI_Datatype t, u;
    int bl[4] = {2, 1, 3, 1}, di[4] = {7, 0, 11, 3};
    MPI_Aint hd[4] = {7 * es, 0, 11 * es, 3 * es};
    int sizes[3] = {5, 6, 7}, subs[3] = {2, 3, 4}, starts[3] = {1, 2, 3};
    int gs[2] = {8, 9}, distr[2] = {MPI_DISTRIBUTE_BLOCK, MPI_DISTRIBUTE_CYCLIC},
        dargs[2] = {MPI_DISTRIBUTE_DFLT_DARG, 2}, psizes[2] = {2, 2};
    ntc = 0;
    MPI_Type_contiguous(5, e, &t); add("contiguous", t, 3);
    MPI_Type_vector(3, 2, 4, e, &t); add("vector", t, 2);
    MPI_Type_create_hvector(4, 1, 3 * es, e, &t); add("hvector", t, 1);
    MPI_Type_indexed(4, bl, di, e, &t); add("indexed", t, 2);
    MPI_Type_create_hindexed(4, bl, hd, e, &t); add("hindexed", t, 1);
    MPI_Type_create_indexed_block(4, 2, di, e, &t); add("indexed_block", t, 1);
    MPI_Type_create_hindexed_block(4, 1, hd, e, &t); add("hindexed_block", t, 2);
    {
        int sbl[3] = {2, 1, 2};
        MPI_Aint sd[3] = {4 * es, -2 * es, 9 * es};
        MPI_Datatype st[3] = {e, e, e};
        MPI_Type_create_struct(3, sbl, sd, st, &t); add("struct_negdisp", t, 1);
    }
    MPI_Type_create_subarray(3, sizes, subs, starts, MPI_ORDER_C, e, &t); add("subarray_c", t, 1);
    MPI_Type_create_subarray(3, sizes, subs, starts, MPI_ORDER_FORTRAN, e, &t); add("subarray_f", t, 1);
    MPI_Type_vector(2, 1, 3, e, &u);
    MPI_Type_create_resized(u, 0, 7 * es, &t); MPI_Type_free(&u); add("resized_vector", t, 3);
    MPI_Type_vector(3, 2, 5, e, &u);
    MPI_Type_create_hvector(2, 1, 17 * es, u, &t); MPI_Type_free(&u); add("vector_of_vector", t, 2);
    MPI_Type_dup(e, &u);
    MPI_Type_vector(2, 3, 4, u, &t); MPI_Type_free(&u); add("vector_of_dup", t, 1);
    MPI_Type_create_darray(4, 3, 2, gs, distr, dargs, psizes, MPI_ORDER_C, e, &t); add("darray", t, 1);
}

static void free_suite(void)
{
    int i;
    for (i = 0; i < ntc; i++) MPI_Type_free(&tc[i].t);
}

/* bytes [lo, hi) a bufcount-copy buffer of t spans, relative to buf */
static void span(MPI_Datatype t, int count, MPI_Aint *lo, MPI_Aint *hi)
{
    MPI_Aint tlb, text, lb, ext;
    MPI_Type_get_true_extent(t, &tlb, &text);
    MPI_Type_get_extent(t, &lb, &ext);
    *lo = tlb < tlb + (count - 1) * ext ? tlb : tlb + (count - 1) * ext;
    *hi = tlb + text > tlb + text + (count - 1) * ext ? tlb + text : tlb + text + (count - 1) * ext;
}

static int check_flatten(void)
{
    static const struct { MPI_Datatype e; int it; const char *n; } el[3] = {
        {MPI_INT, PNCX_ITYPE_INT, "int"}, {MPI_DOUBLE, PNCX_ITYPE_DOUBLE, "double"},
        {MPI_SHORT, PNCX_ITYPE_SHORT, "short"}};
    int k, i, fails = 0;
    for (k = 0; k < 3; k++) {
        int es;
        MPI_Type_size(el[k].e, &es);
        build_suite(el[k].e, es);
        for (i = 0; i < ntc; i++) {
            MPI_Aint lo, hi, lb, ext;
            int size, pos = 0, itype, c;
            MPI_Offset nb, *d, *l, fext, b, j, o = 0, nel = 0;
            unsigned char *buf, *ref, *got;
            int err = pncx_mpi_type_flatten(tc[i].t, &itype, &nb, &d, &l, &fext);
            span(tc[i].t, tc[i].bufcount, &lo, &hi);
            MPI_Type_size(tc[i].t, &size);
            MPI_Type_get_extent(tc[i].t, &lb, &ext);
            buf = (unsigned char *)malloc((size_t)(hi - lo));
            ref = (unsigned char *)malloc((size_t)size * tc[i].bufcount + 1);
            got = (unsigned char *)calloc((size_t)size * tc[i].bufcount + 1, 1);
            for (j = 0; j < hi - lo; j++) buf[j] = (unsigned char)(j * 131 + 7);
            MPI_Pack(buf - lo, tc[i].bufcount, tc[i].t, ref, size * tc[i].bufcount, &pos, MPI_COMM_SELF);
            if (err == NC_NOERR) {
                for (c = 0; c < tc[i].bufcount; c++)
                    for (b = 0; b < nb; b++) {
                        memcpy(got + o, buf - lo + c * fext + d[b], (size_t)(l[b] * es));
                        o += l[b] * es;
                        nel += l[b];
                    }
                free(d);
                free(l);
            }
            if (err != NC_NOERR || itype != el[k].it || fext != ext || o != (MPI_Offset)size * tc[i].bufcount ||
                memcmp(ref, got, (size_t)o) != 0) {
                printf("FAIL flatten %s/%s err=%d itype=%d ext=%lld/%ld bytes=%lld/%d\n", el[k].n, tc[i].name,
                       err, itype, (long long)fext, (long)ext, (long long)o, size * tc[i].bufcount);
                fails++;
            } else {
                printf("ok flatten %s/%s runs=%lld elements=%lld\n", el[k].n, tc[i].name, (long long)nb,
                       (long long)nel);
            }
            free(buf);
            free(ref);
            free(got);
        }
        free_suite();
    }
    /* error codes of ncmpii_dtype_decode */
    {
        MPI_Datatype t, st[2] = {MPI_INT, MPI_DOUBLE};
        int bl[2] = {1, 1}, itype;
        MPI_Aint dd[2] = {0, 8};
        MPI_Offset nb, *d, *l, ext;
        int e1, e2;
        MPI_Type_create_struct(2, bl, dd, st, &t);
        MPI_Type_commit(&t);
        e1 = pncx_mpi_type_flatten(t, &itype, &nb, &d, &l, &ext);
        MPI_Type_free(&t);
        MPI_Type_contiguous(4, MPI_BYTE, &t);
        MPI_Type_commit(&t);
        e2 = pncx_mpi_type_flatten(t, &itype, &nb, &d, &l, &ext);
        MPI_Type_free(&t);
        if (e1 != NC_EMULTITYPES || e2 != NC_EBADTYPE) {
            printf("FAIL error codes: multitypes=%d badtype=%d\n", e1, e2);
            fails++;
        } else {
            printf("ok error codes: NC_EMULTITYPES, NC_EBADTYPE\n");
        }
    }
    return fails;
}

/* ---------------------------------------------------------------- file --- */
typedef struct conv {
    const char *name;
    MPI_Datatype e;
    int xtype;
    int itype;
} conv;

static void fill_values(unsigned char *buf, size_t bytes, MPI_Datatype e, int seed)
{
    size_t i;
    if (e == MPI_DOUBLE) {
        double *p = (double *)buf;
        for (i = 0; i < bytes / 8; i++) p[i] = ((double)((i * 2654435761u + seed) % 200001) - 100000.0) * 0.37;
    } else if (e == MPI_INT) {
        int *p = (int *)buf;
        for (i = 0; i < bytes / 4; i++) p[i] = (int)((i * 2654435761u + seed) % 100001) - 50000;  /* ERANGE for short */
    } else {
        for (i = 0; i < bytes; i++) buf[i] = (unsigned char)(i * 131 + seed);
    }
}

static int read_var_bytes(const char *path, long long off, long long n, unsigned char *out)
{
    FILE *fp = fopen(path, "rb");
    int ok;
    if (fp == NULL) return -1;
    fseek(fp, off, SEEK_SET);
    ok = fread(out, 1, (size_t)n, fp) == (size_t)n;
    fclose(fp);
    return ok ? 0 : -1;
}

static int check_file(const char *dir)
{
    static const conv cv[4] = {
        {"double->NC_DOUBLE", MPI_DOUBLE, NC_DOUBLE, PNCX_ITYPE_DOUBLE},
        {"double->NC_FLOAT", MPI_DOUBLE, NC_FLOAT, PNCX_ITYPE_DOUBLE},
        {"int->NC_SHORT", MPI_INT, NC_SHORT, PNCX_ITYPE_INT},
        {"short->NC_SHORT", MPI_SHORT, NC_SHORT, PNCX_ITYPE_SHORT}};
    int k, i, fails = 0;
    char path[4096];
    for (k = 0; k < 4; k++) {
        int es;
        MPI_Type_size(cv[k].e, &es);
        build_suite(cv[k].e, es);
        for (i = 0; i < ntc; i++) {
            MPI_Aint lo, hi;
            int size, pos, ncid, dim, v0, v1, v2, v3, xs = cv[k].xtype == NC_DOUBLE ? 8 : cv[k].xtype == NC_FLOAT ? 4 : 2;
            int e_flex, e_plain, e_iflex, e_iplain, ids[2], st[2], e_w, e_g1, e_g2, e_ig, e_w2, st2[1];
            MPI_Offset n, start = 0, cnt, o0, o1, o2, o3;
            unsigned char *ubuf, *packed, *fa, *fb, *ga, *gb, *gp;
            size_t ub;
            span(tc[i].t, tc[i].bufcount, &lo, &hi);
            MPI_Type_size(tc[i].t, &size);
            n = (MPI_Offset)size / es * tc[i].bufcount;
            cnt = n;
            ub = (size_t)(hi - lo);
            ubuf = (unsigned char *)malloc(ub);
            packed = (unsigned char *)malloc((size_t)size * tc[i].bufcount);
            fa = (unsigned char *)malloc((size_t)n * xs);
            fb = (unsigned char *)malloc((size_t)n * xs);
            ga = (unsigned char *)malloc(ub);
            gb = (unsigned char *)malloc(ub);
            gp = (unsigned char *)malloc((size_t)size * tc[i].bufcount);
            fill_values(ubuf, ub, cv[k].e, 11 * i + k);
            pos = 0;
            MPI_Pack(ubuf - lo, tc[i].bufcount, tc[i].t, packed, size * tc[i].bufcount, &pos, MPI_COMM_SELF);
            snprintf(path, sizeof path, "%s/flex_%d_%d.nc", dir, k, i);
            pncx_nc_create(path, NC_64BIT_DATA, &ncid);
            pncx_nc_def_dim(ncid, "n", n, &dim);
            pncx_nc_def_var(ncid, "flex", cv[k].xtype, 1, &dim, &v0);
            pncx_nc_def_var(ncid, "plain", cv[k].xtype, 1, &dim, &v1);
            pncx_nc_def_var(ncid, "iflex", cv[k].xtype, 1, &dim, &v2);
            pncx_nc_def_var(ncid, "iplain", cv[k].xtype, 1, &dim, &v3);
            pncx_nc_enddef(ncid);
            /* put: derived type vs MPI_Pack + contiguous (the reference's order of work) */
            e_flex = pncx_ncmpi_put_varm(ncid, v0, &start, &cnt, NULL, NULL, ubuf - lo, tc[i].bufcount, tc[i].t);
            e_plain = pncx_ncmpi_put_varm(ncid, v1, &start, &cnt, NULL, NULL, packed, NC_COUNT_IGNORE, cv[k].e);
            e_iflex = pncx_ncmpi_iput_varm(ncid, v2, &start, &cnt, NULL, NULL, ubuf - lo, tc[i].bufcount, tc[i].t, &ids[0]);
            e_iplain = pncx_ncmpi_iput_varm(ncid, v3, &start, &cnt, NULL, NULL, packed, NC_COUNT_IGNORE, cv[k].e, &ids[1]);
            e_w = pncx_nc_wait_all(ncid, 2, ids, st);
            /* get: derived type into a sentinel buffer vs contiguous get + MPI_Unpack */
            memset(ga, 0xA5, ub);
            memset(gb, 0xA5, ub);
            e_g1 = pncx_ncmpi_get_varm(ncid, v0, &start, &cnt, NULL, NULL, ga - lo, tc[i].bufcount, tc[i].t);
            e_g2 = pncx_ncmpi_get_varm(ncid, v0, &start, &cnt, NULL, NULL, gp, NC_COUNT_IGNORE, cv[k].e);
            pos = 0;
            MPI_Unpack(gp, size * tc[i].bufcount, &pos, gb - lo, tc[i].bufcount, tc[i].t, MPI_COMM_SELF);
            {
                int ok = memcmp(ga, gb, ub) == 0, okb, oki, okig;
                unsigned char *gi = (unsigned char *)malloc(ub);
                memset(gi, 0xA5, ub);
                e_ig = pncx_ncmpi_iget_varm(ncid, v2, &start, &cnt, NULL, NULL, gi - lo, tc[i].bufcount, tc[i].t, &ids[0]);
                e_w2 = pncx_nc_wait_all(ncid, 1, ids, st2);
                okig = memcmp(gi, gb, ub) == 0;
                free(gi);
                pncx_nc_inq_varoffset(ncid, v0, &o0);
                pncx_nc_inq_varoffset(ncid, v1, &o1);
                pncx_nc_inq_varoffset(ncid, v2, &o2);
                pncx_nc_inq_varoffset(ncid, v3, &o3);
                pncx_nc_close(ncid);
                okb = read_var_bytes(path, o0, n * xs, fa) == 0 && read_var_bytes(path, o1, n * xs, fb) == 0 &&
                      memcmp(fa, fb, (size_t)(n * xs)) == 0;
                oki = read_var_bytes(path, o2, n * xs, fa) == 0 && read_var_bytes(path, o3, n * xs, fb) == 0 &&
                      memcmp(fa, fb, (size_t)(n * xs)) == 0;
                if (!okb || !oki || !ok || !okig || e_flex != e_plain || e_iflex != NC_NOERR ||
                    e_iplain != NC_NOERR || e_w != (st[0] ? st[0] : st[1]) || st[0] != st[1] ||
                    e_g1 != e_g2 || e_ig != NC_NOERR || e_w2 != st2[0] || st2[0] != e_g2) {
                    printf("FAIL file %s/%s put_bytes=%d iput_bytes=%d get=%d iget=%d status put %d/%d iput %d/%d "
                           "get %d/%d iget %d\n", cv[k].name, tc[i].name, okb, oki, ok, okig, e_flex, e_plain,
                           st[0], st[1], e_g1, e_g2, st2[0]);
                    fails++;
                } else {
                    printf("ok file %s/%s n=%lld status=%d\n", cv[k].name, tc[i].name, (long long)n, e_flex);
                }
            }
            remove(path);
            free(ubuf); free(packed); free(fa); free(fb); free(ga); free(gb); free(gp);
        }
        free_suite();
    }
    return fails;
}

int main(int argc, char **argv)
{
    int fails;
    MPI_Init(&argc, &argv);
    if (argc >= 2 && strcmp(argv[1], "flatten") == 0) fails = check_flatten();
    else if (argc >= 3 && strcmp(argv[1], "file") == 0) {
        if (pncx_device_count() <= 0) { printf("FAIL file: no GPU visible\n"); fails = 1; }
        else fails = check_file(argv[2]);
    }
    else { fprintf(stderr, "usage: flex_check flatten | file <dir>\n"); fails = 1; }
    printf("%s: %d failure(s)\n", argc >= 2 ? argv[1] : "?", fails);
    MPI_Finalize();
    return fails ? 1 : 0;
}
