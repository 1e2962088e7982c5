/*
 * pncx_mpi.c -- MPI derived buftypes for the flexible API (include/pncx_mpi.h).
 *
 * The reference decodes a buftype with ncmpii_dtype_decode
 * (src/drivers/common/dtype_decode.c:89-399: element type, element count,
 * NC_EMULTITYPES) and moves the data with MPI_Pack/MPI_Unpack
 * (ncmpio_util.c:620-652, 889-933).  Here the datatype's typemap is
 * flattened once into runs of elements (pack order, byte displacements from
 * the buffer origin) and committed; the GPU kernels then gather/scatter it
 * fused with the conversion.  Host-only code: no device work happens here
 * except through pncx_type_commit.
 */
#include <stdlib.h>
#include <string.h>

#include "../../include/pncx_mpi.h"
#include "../../include/pncx_ncmpii.h"

typedef struct blist {
    long long n, cap;
    long long *disp, *len;
} blist;

typedef struct fctx {
    int itype;      /* element type seen so far (0 = none yet) */
    int esize;
} fctx;

static void bl_free(blist *b)
{
    free(b->disp);
    free(b->len);
    memset(b, 0, sizeof *b);
}

/* append a run, merging it into the previous run when it continues it */
static int bl_add(blist *b, const fctx *c, long long disp, long long len)
{
    if (len <= 0) return NC_NOERR;
    if (b->n > 0 && b->disp[b->n - 1] + b->len[b->n - 1] * c->esize == disp) {
        b->len[b->n - 1] += len;
        return NC_NOERR;
    }
    if (b->n == b->cap) {
        const long long cap = b->cap ? 2 * b->cap : 16;
        long long *d = (long long *)realloc(b->disp, sizeof(long long) * (size_t)cap);
        long long *l;
        if (d == NULL) return NC_ENOMEM;
        b->disp = d;
        l = (long long *)realloc(b->len, sizeof(long long) * (size_t)cap);
        if (l == NULL) return NC_ENOMEM;
        b->len = l;
        b->cap = cap;
    }
    b->disp[b->n] = disp;
    b->len[b->n] = len;
    b->n++;
    return NC_NOERR;
}

/* append `count` copies of sub, copy k at off + k*ext */
static int bl_rep(blist *out, const fctx *c, const blist *sub, long long off, long long count, long long ext)
{
    long long k, i;
    int err = NC_NOERR;
    if (sub->n == 1 && sub->len[0] * c->esize == ext)       /* contiguous copies: one run */
        return bl_add(out, c, off + sub->disp[0], sub->len[0] * count);
    for (k = 0; k < count && !err; k++)
        for (i = 0; i < sub->n && !err; i++) err = bl_add(out, c, off + k * ext + sub->disp[i], sub->len[i]);
    return err;
}

static long long type_extent(MPI_Datatype t)
{
    MPI_Aint lb, ext;
    MPI_Type_get_extent(t, &lb, &ext);
    return (long long)ext;
}

static int flat(MPI_Datatype t, fctx *c, blist *out);

/* typemap of one copy of t into a fresh list */
static int flat_sub(MPI_Datatype t, fctx *c, blist *sub)
{
    memset(sub, 0, sizeof *sub);
    return flat(t, c, sub);
}

/*
 * Combiners the flattening has no rule for (darray, f90 types): MPI_Pack
 * itself says where every packed byte comes from.  Plane p of a scratch
 * buffer holds byte p of each byte's own offset; packing it and reading the
 * first byte of every packed element gives that element's offset, one byte
 * at a time.  The element type comes from the combiner's old type.
 */
static int flat_by_pack(MPI_Datatype t, MPI_Datatype old, fctx *c, blist *out)
{
    MPI_Aint tlb, text;
    int size, p, planes = 1, pos, err = NC_NOERR;
    long long k, nel, i;
    unsigned char *src = NULL, *packed = NULL;
    long long *offs = NULL;
    blist sub;
    if (old == MPI_DATATYPE_NULL) return NC_EBADTYPE;
    if ((err = flat_sub(old, c, &sub)) != NC_NOERR) { bl_free(&sub); return err; }
    bl_free(&sub);
    MPI_Type_get_true_extent(t, &tlb, &text);
    MPI_Type_size(t, &size);
    if (size == 0) return NC_NOERR;
    if (c->esize <= 0) return NC_EBADTYPE;
    while (planes < 8 && ((unsigned long long)(text - 1) >> (8 * planes)) != 0) planes++;
    nel = size / c->esize;
    src = (unsigned char *)malloc((size_t)text);
    packed = (unsigned char *)malloc((size_t)size);
    offs = (long long *)calloc((size_t)nel, sizeof(long long));
    if (src == NULL || packed == NULL || offs == NULL) { err = NC_ENOMEM; goto out; }
    for (p = 0; p < planes; p++) {
        for (i = 0; i < text; i++) src[i] = (unsigned char)((unsigned long long)i >> (8 * p));
        pos = 0;
        if (MPI_Pack(src - tlb, 1, t, packed, size, &pos, MPI_COMM_SELF) != MPI_SUCCESS) { err = NC_EINVAL; goto out; }
        for (k = 0; k < nel; k++) offs[k] |= (long long)packed[k * c->esize] << (8 * p);
    }
    for (k = 0; k < nel && !err; k++) err = bl_add(out, c, offs[k] + tlb, 1);
out:
    free(src);
    free(packed);
    free(offs);
    return err;
}

static void free_types(MPI_Datatype *types, int nd)
{
    int i, ni, na, ndt, comb;
    for (i = 0; i < nd; i++) {
        MPI_Type_get_envelope(types[i], &ni, &na, &ndt, &comb);
        if (comb != MPI_COMBINER_NAMED) MPI_Type_free(&types[i]);
    }
}

/* typemap of one copy of t, relative to its origin, appended to out
 * (the combiner cases of ncmpii_dtype_decode, dtype_decode.c:198-399) */
static int flat(MPI_Datatype t, fctx *c, blist *out)
{
    int ni, na, nd, comb, err = NC_NOERR, i;
    int *ints = NULL;
    MPI_Aint *addrs = NULL;
    MPI_Datatype *types = NULL;
    blist sub;
    long long k, ext;
    memset(&sub, 0, sizeof sub);
    if (t == MPI_DATATYPE_NULL) return NC_EINVAL;
    MPI_Type_get_envelope(t, &ni, &na, &nd, &comb);
    if (comb == MPI_COMBINER_NAMED) {
        const int it = pncx_itype_from_mpi(t);
        if (it == 0) return NC_EBADTYPE;              /* MPI_BYTE, MPI_LONG_DOUBLE, ... */
        if (c->itype == 0) {
            c->itype = it;
            c->esize = pncx_ilen(it);
        } else if (c->itype != it) {
            return NC_EMULTITYPES;                    /* dtype_decode.c:272 */
        }
        return bl_add(out, c, 0, 1);
    }
    ints = (int *)malloc(sizeof(int) * (size_t)(ni ? ni : 1));
    addrs = (MPI_Aint *)malloc(sizeof(MPI_Aint) * (size_t)(na ? na : 1));
    types = (MPI_Datatype *)malloc(sizeof(MPI_Datatype) * (size_t)(nd ? nd : 1));
    if (ints == NULL || addrs == NULL || types == NULL) { err = NC_ENOMEM; goto out0; }
    MPI_Type_get_contents(t, ni, na, nd, ints, addrs, types);
    switch (comb) {
        case MPI_COMBINER_DUP:
        case MPI_COMBINER_RESIZED:          /* one copy: the old typemap; only the extent differs */
            err = flat(types[0], c, out);
            break;
        case MPI_COMBINER_CONTIGUOUS:
            if ((err = flat_sub(types[0], c, &sub)) == NC_NOERR)
                err = bl_rep(out, c, &sub, 0, ints[0], type_extent(types[0]));
            break;
        case MPI_COMBINER_VECTOR:
        case MPI_COMBINER_HVECTOR:
        case MPI_COMBINER_HVECTOR_INTEGER: {
            long long stride;
            ext = type_extent(types[0]);
            stride = comb == MPI_COMBINER_VECTOR ? (long long)ints[2] * ext
                   : comb == MPI_COMBINER_HVECTOR ? (long long)addrs[0] : (long long)ints[2];
            if ((err = flat_sub(types[0], c, &sub)) == NC_NOERR)
                for (k = 0; k < ints[0] && !err; k++) err = bl_rep(out, c, &sub, k * stride, ints[1], ext);
            break;
        }
        case MPI_COMBINER_INDEXED:
        case MPI_COMBINER_HINDEXED:
        case MPI_COMBINER_HINDEXED_INTEGER: {
            const int n = ints[0];
            ext = type_extent(types[0]);
            if ((err = flat_sub(types[0], c, &sub)) == NC_NOERR)
                for (i = 0; i < n && !err; i++) {
                    const long long d = comb == MPI_COMBINER_INDEXED ? (long long)ints[1 + n + i] * ext
                                      : comb == MPI_COMBINER_HINDEXED ? (long long)addrs[i]
                                                                      : (long long)ints[1 + n + i];
                    err = bl_rep(out, c, &sub, d, ints[1 + i], ext);
                }
            break;
        }
        case MPI_COMBINER_INDEXED_BLOCK:
        case MPI_COMBINER_HINDEXED_BLOCK: {
            const int n = ints[0];
            ext = type_extent(types[0]);
            if ((err = flat_sub(types[0], c, &sub)) == NC_NOERR)
                for (i = 0; i < n && !err; i++) {
                    const long long d = comb == MPI_COMBINER_INDEXED_BLOCK ? (long long)ints[2 + i] * ext
                                                                          : (long long)addrs[i];
                    err = bl_rep(out, c, &sub, d, ints[1], ext);
                }
            break;
        }
        case MPI_COMBINER_STRUCT:
        case MPI_COMBINER_STRUCT_INTEGER: {
            const int n = ints[0];
            for (i = 0; i < n && !err; i++) {
                const long long d = comb == MPI_COMBINER_STRUCT ? (long long)addrs[i] : (long long)ints[1 + n + i];
                blist si;
                if ((err = flat_sub(types[i], c, &si)) == NC_NOERR)
                    err = bl_rep(out, c, &si, d, ints[1 + i], type_extent(types[i]));
                bl_free(&si);
            }
            break;
        }
        case MPI_COMBINER_SUBARRAY: {
            /* ints: ndims, sizes[], subsizes[], starts[], order */
            const int n = ints[0];
            const int *sizes = ints + 1, *subs = ints + 1 + n, *starts = ints + 1 + 2 * n;
            const int forder = ints[1 + 3 * n] == MPI_ORDER_FORTRAN;
            long long stride[32], idx[32], total = 1, base = 0;
            int d;
            if (n > 32) { err = NC_EINVAL; break; }
            ext = type_extent(types[0]);
            if ((err = flat_sub(types[0], c, &sub)) != NC_NOERR) break;
            /* element strides, fastest dimension last (C) or first (Fortran) */
            for (d = 0; d < n; d++) {
                const int dd = forder ? d : n - 1 - d;
                stride[dd] = d == 0 ? ext : stride[forder ? dd - 1 : dd + 1] * sizes[forder ? dd - 1 : dd + 1];
            }
            for (d = 0; d < n; d++) {
                total *= subs[d];
                idx[d] = 0;
                base += (long long)starts[d] * stride[d];
            }
            if (total == 0) break;
            {
                const int fast = forder ? 0 : n - 1;     /* innermost dimension: one run of copies */
                for (;;) {
                    long long off = base;
                    for (d = 0; d < n; d++) off += idx[d] * stride[d];
                    if ((err = bl_rep(out, c, &sub, off, subs[fast], ext)) != NC_NOERR) break;
                    /* odometer over the other dimensions */
                    for (d = forder ? 1 : n - 2; forder ? d < n : d >= 0; d += forder ? 1 : -1) {
                        if (++idx[d] < subs[d]) break;
                        idx[d] = 0;
                    }
                    if (forder ? d == n : d < 0) break;
                }
            }
            break;
        }
        default:                            /* darray, f90 types, ... */
            err = flat_by_pack(t, nd > 0 ? types[nd - 1] : MPI_DATATYPE_NULL, c, out);
            break;
    }
    bl_free(&sub);
    free_types(types, nd);
out0:
    free(ints);
    free(addrs);
    free(types);
    return err;
}

int pncx_mpi_type_flatten(MPI_Datatype buftype, int *itype, MPI_Offset *nblocks, MPI_Offset **disp,
                          MPI_Offset **blocklen, MPI_Offset *extent)
{
    fctx c = {0, 1};
    blist out;
    int err;
    memset(&out, 0, sizeof out);
    if (itype == NULL || nblocks == NULL || disp == NULL || blocklen == NULL || extent == NULL)
        return NC_EINVAL;
    err = flat(buftype, &c, &out);
    if (err != NC_NOERR) { bl_free(&out); return err; }
    *itype = c.itype ? c.itype : PNCX_ITYPE_UCHAR;     /* an empty type carries no elements */
    *nblocks = out.n;
    *disp = out.disp;
    *blocklen = out.len;
    *extent = type_extent(buftype);
    return NC_NOERR;
}

int pncx_mpi_type_commit(MPI_Datatype buftype, pncx_dtype **dtype)
{
    int itype, err;
    MPI_Offset n, *d, *l, ext;
    if ((err = pncx_mpi_type_flatten(buftype, &itype, &n, &d, &l, &ext)) != NC_NOERR) return err;
    err = pncx_type_commit(itype, n, d, l, ext, dtype);
    free(d);
    free(l);
    return err;
}

/* ---- the flexible ncmpi_{put,get,iput,iget}_varm ---- */
enum { K_PUT, K_GET, K_IPUT, K_IGET };

static int flex(int kind, int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                const MPI_Offset *stride, const MPI_Offset *imap, void *buf, MPI_Offset bufcount,
                MPI_Datatype buftype, int *reqid)
{
    pncx_dtype *dt = NULL;
    int err;
    if (buftype != MPI_DATATYPE_NULL && bufcount == NC_COUNT_IGNORE) {
        /* high-level API: a predefined type (var_getput.m4:366-377) */
        const int it = pncx_itype_from_mpi(buftype);
        if (it == 0) return NC_EINVAL;
        switch (kind) {
            case K_PUT: return pncx_nc_put_varm(ncid, varid, start, count, stride, imap, buf, it);
            case K_GET: return pncx_nc_get_varm(ncid, varid, start, count, stride, imap, buf, it);
            case K_IPUT: return pncx_nc_iput_varm(ncid, varid, start, count, stride, imap, buf, it, reqid);
            default: return pncx_nc_iget_varm(ncid, varid, start, count, stride, imap, buf, it, reqid);
        }
    }
    if (buftype != MPI_DATATYPE_NULL && (err = pncx_mpi_type_commit(buftype, &dt)) != NC_NOERR) return err;
    switch (kind) {
        case K_PUT: err = pncx_nc_put_varm_flex(ncid, varid, start, count, stride, imap, buf, bufcount, dt); break;
        case K_GET: err = pncx_nc_get_varm_flex(ncid, varid, start, count, stride, imap, buf, bufcount, dt); break;
        case K_IPUT: err = pncx_nc_iput_varm_flex(ncid, varid, start, count, stride, imap, buf, bufcount, dt, reqid); break;
        default: err = pncx_nc_iget_varm_flex(ncid, varid, start, count, stride, imap, buf, bufcount, dt, reqid); break;
    }
    if (dt != NULL) pncx_type_free(dt);      /* a posted request keeps its own reference */
    return err;
}

int pncx_ncmpi_put_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                        const MPI_Offset *stride, const MPI_Offset *imap, const void *buf,
                        MPI_Offset bufcount, MPI_Datatype buftype)
{
    return flex(K_PUT, ncid, varid, start, count, stride, imap, (void *)buf, bufcount, buftype, NULL);
}

int pncx_ncmpi_get_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                        const MPI_Offset *stride, const MPI_Offset *imap, void *buf,
                        MPI_Offset bufcount, MPI_Datatype buftype)
{
    return flex(K_GET, ncid, varid, start, count, stride, imap, buf, bufcount, buftype, NULL);
}

int pncx_ncmpi_iput_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                         const MPI_Offset *stride, const MPI_Offset *imap, const void *buf,
                         MPI_Offset bufcount, MPI_Datatype buftype, int *reqid)
{
    return flex(K_IPUT, ncid, varid, start, count, stride, imap, (void *)buf, bufcount, buftype, reqid);
}

int pncx_ncmpi_iget_varm(int ncid, int varid, const MPI_Offset *start, const MPI_Offset *count,
                         const MPI_Offset *stride, const MPI_Offset *imap, void *buf,
                         MPI_Offset bufcount, MPI_Datatype buftype, int *reqid)
{
    return flex(K_IGET, ncid, varid, start, count, stride, imap, buf, bufcount, buftype, reqid);
}
