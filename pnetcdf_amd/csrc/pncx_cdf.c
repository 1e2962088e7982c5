/*
 * pncx_cdf.c -- classic CDF-1/2/5 header codec and variable layout.
 *
 * Host C, no device work: the header is a few hundred bytes to a few MB and
 * is parsed once per open.  Behaviour follows the reference:
 *   length      ncmpio_header_get.c:128-322,1273-1311 (hdr_len_NC_*)
 *   encode      ncmpio_header_put.c:32-592          (hdr_put_NC_*)
 *   decode      ncmpio_header_get.c:418-1271,1327-1445 (hdr_get_NC_*),
 *               including its error order: NC_ENOTNC for a bad magic or list
 *               tag, NC_EMAXDIMS / NC_EMAXATTS / NC_EMAXVARS for counts above
 *               NC_MAX_INT, NC_EMAXNAME, NC_EBADTYPE, NC_EBADDIM, NC_EUNLIMIT,
 *               NC_ENULLPAD (non fatal, ncvalidator mode only)
 *   shape       ncmpio_var.c:282-355                (ncmpio_NC_var_shape64)
 *   shape check ncmpio_header_get.c:34-97           (compute_var_shape)
 *   size check  ncmpio_enddef.c:785-897             (ncmpio_NC_check_vlen[s])
 *   begins      ncmpio_enddef.c:359-612             (NC_begins)
 *   offsets     ncmpio_enddef.c:950-1117            (ncmpio_NC_check_voffs)
 *   names       drivers/common/check_name.c:196-243 (check_name_CDF2)
 */
#include <stdlib.h>
#include <string.h>

#include "pncx.h"
#include "pncx_nc.h"
#include "pncx_cdf.h"

#define RNDUP(x, a) ((((x) + (a) - 1) / (a)) * (a))

static int xlen_of(int xtype) { return pncx_xlen(xtype); }

/* ------------------------------------------------------------------------ */
/* object lifetime                                                          */
/* ------------------------------------------------------------------------ */
void cdf_hdr_init(cdf_hdr *h, int format)
{
    memset(h, 0, sizeof *h);
    h->format = format;
    h->unlimited_id = -1;
    h->h_minfree = 0;
    h->v_minfree = 0;
    h->v_align = 0;
    h->r_align = 0;
}

static void atts_free(cdf_atts *a)
{
    int i;
    for (i = 0; i < a->n; i++) {
        free(a->v[i].name);
        free(a->v[i].xvalue);
    }
    free(a->v);
    memset(a, 0, sizeof *a);
}

static void var_free(cdf_var *v)
{
    free(v->name);
    free(v->dimids);
    free(v->shape);
    free(v->dsizes);
    atts_free(&v->atts);
}

void cdf_hdr_free(cdf_hdr *h)
{
    int i;
    for (i = 0; i < h->ndims; i++) free(h->dims[i].name);
    free(h->dims);
    atts_free(&h->gatts);
    for (i = 0; i < h->nvars; i++) var_free(&h->vars[i]);
    free(h->vars);
    memset(h, 0, sizeof *h);
    h->unlimited_id = -1;
}

static char *dupstr(const char *s, size_t n)
{
    char *d = (char *)malloc(n + 1);
    if (d == NULL) return NULL;
    memcpy(d, s, n);
    d[n] = '\0';
    return d;
}

static int atts_copy(cdf_atts *d, const cdf_atts *s)
{
    int i;
    memset(d, 0, sizeof *d);
    if (s->n == 0) return NC_NOERR;
    d->v = (cdf_att *)calloc((size_t)s->n, sizeof(cdf_att));
    if (d->v == NULL) return NC_ENOMEM;
    d->cap = d->n = s->n;
    for (i = 0; i < s->n; i++) {
        d->v[i] = s->v[i];
        d->v[i].name = dupstr(s->v[i].name, strlen(s->v[i].name));
        d->v[i].xvalue = (unsigned char *)malloc((size_t)(s->v[i].xsz ? s->v[i].xsz : 1));
        if (d->v[i].name == NULL || d->v[i].xvalue == NULL) return NC_ENOMEM;
        memcpy(d->v[i].xvalue, s->v[i].xvalue, (size_t)s->v[i].xsz);
    }
    return NC_NOERR;
}

int cdf_hdr_copy(cdf_hdr *d, const cdf_hdr *s)
{
    int i, err;
    *d = *s;
    d->dims = NULL;
    d->vars = NULL;
    d->capd = s->ndims;
    d->capv = s->nvars;
    if (s->ndims) {
        d->dims = (cdf_dim *)calloc((size_t)s->ndims, sizeof(cdf_dim));
        if (d->dims == NULL) return NC_ENOMEM;
        for (i = 0; i < s->ndims; i++) {
            d->dims[i].size = s->dims[i].size;
            d->dims[i].name = dupstr(s->dims[i].name, strlen(s->dims[i].name));
            if (d->dims[i].name == NULL) return NC_ENOMEM;
        }
    }
    if ((err = atts_copy(&d->gatts, &s->gatts)) != NC_NOERR) return err;
    if (s->nvars) {
        d->vars = (cdf_var *)calloc((size_t)s->nvars, sizeof(cdf_var));
        if (d->vars == NULL) return NC_ENOMEM;
        for (i = 0; i < s->nvars; i++) {
            const cdf_var *sv = &s->vars[i];
            cdf_var *dv = &d->vars[i];
            const size_t nd = (size_t)(sv->ndims ? sv->ndims : 1);
            *dv = *sv;
            dv->name = dupstr(sv->name, strlen(sv->name));
            dv->dimids = (int *)calloc(nd, sizeof(int));
            dv->shape = (long long *)calloc(nd, sizeof(long long));
            dv->dsizes = (long long *)calloc(nd, sizeof(long long));
            if (!dv->name || !dv->dimids || !dv->shape || !dv->dsizes) return NC_ENOMEM;
            memcpy(dv->dimids, sv->dimids, sizeof(int) * (size_t)sv->ndims);
            memcpy(dv->shape, sv->shape, sizeof(long long) * (size_t)sv->ndims);
            memcpy(dv->dsizes, sv->dsizes, sizeof(long long) * (size_t)sv->ndims);
            if ((err = atts_copy(&dv->atts, &sv->atts)) != NC_NOERR) return err;
        }
    }
    return NC_NOERR;
}

/* ------------------------------------------------------------------------ */
/* names, lookup, definition                                                */
/* ------------------------------------------------------------------------ */
/* UTF-8 sequence length starting at p, or -1 when malformed */
static int utf8_len(const unsigned char *p)
{
    int n, i;
    if (p[0] < 0x80) return 1;
    if ((p[0] & 0xE0) == 0xC0) n = 2;
    else if ((p[0] & 0xF0) == 0xE0) n = 3;
    else if ((p[0] & 0xF8) == 0xF0) n = 4;
    else return -1;
    for (i = 1; i < n; i++)
        if ((p[i] & 0xC0) != 0x80) return -1;
    return n;
}

int cdf_check_name(const char *name)
{
    const unsigned char *cp = (const unsigned char *)name;
    unsigned char ch;
    int skip;
    if (name == NULL || *name == 0 || strchr(name, '/')) return NC_EBADNAME;
    if (strlen(name) > CDF_MAX_NAME) return NC_EMAXNAME;
    ch = *cp;
    if (ch <= 0x7f) {
        if (!((ch >= 'A' && ch <= 'Z') || (ch >= 'a' && ch <= 'z') || (ch >= '0' && ch <= '9') || ch == '_'))
            return NC_EBADNAME;
        cp++;
    } else {
        if ((skip = utf8_len(cp)) < 0) return NC_EBADNAME;
        cp += skip;
    }
    while (*cp) {
        ch = *cp;
        if (ch <= 0x7f) {
            if (ch < ' ' || ch > 0x7E) return NC_EBADNAME;
            cp++;
        } else {
            if ((skip = utf8_len(cp)) < 0) return NC_EBADNAME;
            cp += skip;
        }
    }
    if (ch <= 0x7f && (ch == ' ' || (ch >= '\t' && ch <= '\r'))) return NC_EBADNAME;   /* trailing space */
    return NC_NOERR;
}

int cdf_find_dim(const cdf_hdr *h, const char *name)
{
    int i;
    for (i = 0; i < h->ndims; i++)
        if (strcmp(h->dims[i].name, name) == 0) return i;
    return -1;
}

int cdf_find_var(const cdf_hdr *h, const char *name)
{
    int i;
    for (i = 0; i < h->nvars; i++)
        if (strcmp(h->vars[i].name, name) == 0) return i;
    return -1;
}

int cdf_find_att(const cdf_atts *a, const char *name)
{
    int i;
    for (i = 0; i < a->n; i++)
        if (strcmp(a->v[i].name, name) == 0) return i;
    return -1;
}

int cdf_add_dim(cdf_hdr *h, const char *name, long long size)
{
    if (h->ndims == h->capd) {
        const int cap = h->capd ? 2 * h->capd : 16;
        cdf_dim *d = (cdf_dim *)realloc(h->dims, sizeof(cdf_dim) * (size_t)cap);
        if (d == NULL) return NC_ENOMEM;
        h->dims = d;
        h->capd = cap;
    }
    h->dims[h->ndims].name = dupstr(name, strlen(name));
    if (h->dims[h->ndims].name == NULL) return NC_ENOMEM;
    h->dims[h->ndims].size = size;
    if (size == 0) h->unlimited_id = h->ndims;
    h->ndims++;
    return NC_NOERR;
}

int cdf_add_var(cdf_hdr *h, const char *name, int xtype, int ndims, const int *dimids)
{
    cdf_var *v;
    const size_t nd = (size_t)(ndims ? ndims : 1);
    if (h->nvars == h->capv) {
        const int cap = h->capv ? 2 * h->capv : 16;
        cdf_var *nv = (cdf_var *)realloc(h->vars, sizeof(cdf_var) * (size_t)cap);
        if (nv == NULL) return NC_ENOMEM;
        h->vars = nv;
        h->capv = cap;
    }
    v = &h->vars[h->nvars];
    memset(v, 0, sizeof *v);
    v->name = dupstr(name, strlen(name));
    v->dimids = (int *)calloc(nd, sizeof(int));
    v->shape = (long long *)calloc(nd, sizeof(long long));
    v->dsizes = (long long *)calloc(nd, sizeof(long long));
    if (!v->name || !v->dimids || !v->shape || !v->dsizes) { var_free(v); return NC_ENOMEM; }
    v->ndims = ndims;
    if (ndims && dimids) memcpy(v->dimids, dimids, sizeof(int) * (size_t)ndims);
    v->xtype = xtype;
    v->xsz = xlen_of(xtype);
    h->nvars++;
    return NC_NOERR;
}

int cdf_set_att(cdf_atts *a, const char *name, int xtype, long long nelems, const void *xvalue)
{
    const int xl = xlen_of(xtype);
    const long long nbytes = nelems * xl, xsz = RNDUP(nbytes, 4);
    int i = cdf_find_att(a, name);
    unsigned char *val;
    if (xl < 0) return NC_EBADTYPE;
    if (nelems < 0) return NC_EINVAL;
    val = (unsigned char *)calloc(1, (size_t)(xsz ? xsz : 1));
    if (val == NULL) return NC_ENOMEM;
    if (nbytes) memcpy(val, xvalue, (size_t)nbytes);
    if (i < 0) {
        if (a->n == a->cap) {
            const int cap = a->cap ? 2 * a->cap : 8;
            cdf_att *nv = (cdf_att *)realloc(a->v, sizeof(cdf_att) * (size_t)cap);
            if (nv == NULL) { free(val); return NC_ENOMEM; }
            a->v = nv;
            a->cap = cap;
        }
        i = a->n++;
        a->v[i].name = dupstr(name, strlen(name));
        if (a->v[i].name == NULL) { a->n--; free(val); return NC_ENOMEM; }
    } else {
        free(a->v[i].xvalue);
    }
    a->v[i].xtype = xtype;
    a->v[i].nelems = nelems;
    a->v[i].xsz = xsz;
    a->v[i].xvalue = val;
    return NC_NOERR;
}

int cdf_del_att(cdf_atts *a, const char *name)
{
    const int i = cdf_find_att(a, name);
    if (i < 0) return NC_ENOTATT;
    free(a->v[i].name);
    free(a->v[i].xvalue);
    memmove(&a->v[i], &a->v[i + 1], sizeof(cdf_att) * (size_t)(a->n - i - 1));
    a->n--;
    return NC_NOERR;
}

/* ------------------------------------------------------------------------ */
/* header length and encoding                                               */
/* ------------------------------------------------------------------------ */
static long long atts_len(const cdf_atts *a, int nn)
{
    long long x = 4 + nn;
    int i;
    for (i = 0; i < a->n; i++)
        x += nn + RNDUP((long long)strlen(a->v[i].name), 4) + 4 + nn + a->v[i].xsz;
    return x;
}

long long cdf_hdr_len(const cdf_hdr *h)
{
    const int nn = h->format == 5 ? 8 : 4, off = h->format == 1 ? 4 : 8;
    long long x = 4 + nn;
    int i;
    x += 4 + nn;
    for (i = 0; i < h->ndims; i++) x += nn + RNDUP((long long)strlen(h->dims[i].name), 4) + nn;
    x += atts_len(&h->gatts, nn);
    x += 4 + nn;
    for (i = 0; i < h->nvars; i++) {
        const cdf_var *v = &h->vars[i];
        x += nn + RNDUP((long long)strlen(v->name), 4) + nn + (long long)nn * v->ndims +
             atts_len(&v->atts, nn) + 4 + nn + off;
    }
    return x;
}

typedef struct wbuf { unsigned char *p; int nn; } wbuf;

static void put_u32(wbuf *w, unsigned long long v)
{
    w->p[0] = (unsigned char)(v >> 24);
    w->p[1] = (unsigned char)(v >> 16);
    w->p[2] = (unsigned char)(v >> 8);
    w->p[3] = (unsigned char)v;
    w->p += 4;
}

static void put_u64(wbuf *w, unsigned long long v)
{
    put_u32(w, v >> 32);
    put_u32(w, v & 0xFFFFFFFFull);
}

static void put_nn(wbuf *w, unsigned long long v) { if (w->nn == 8) put_u64(w, v); else put_u32(w, v); }

static void put_name(wbuf *w, const char *s)
{
    const size_t n = strlen(s), pad = (size_t)RNDUP((long long)n, 4) - n;
    put_nn(w, n);
    memcpy(w->p, s, n);
    memset(w->p + n, 0, pad);
    w->p += n + pad;
}

static void put_atts(wbuf *w, const cdf_atts *a)
{
    int i;
    if (a->n == 0) {                      /* ABSENT = ZERO ZERO[64] */
        put_u32(w, 0);
        put_nn(w, 0);
        return;
    }
    put_u32(w, CDF_ATTRIBUTE);
    put_nn(w, (unsigned long long)a->n);
    for (i = 0; i < a->n; i++) {
        put_name(w, a->v[i].name);
        put_u32(w, (unsigned long long)a->v[i].xtype);
        put_nn(w, (unsigned long long)a->v[i].nelems);
        memcpy(w->p, a->v[i].xvalue, (size_t)a->v[i].xsz);   /* already zero padded */
        w->p += a->v[i].xsz;
    }
}

long long cdf_hdr_encode(const cdf_hdr *h, unsigned char *buf)
{
    wbuf w;
    int i, d;
    w.p = buf;
    w.nn = h->format == 5 ? 8 : 4;
    w.p[0] = 'C'; w.p[1] = 'D'; w.p[2] = 'F'; w.p[3] = (unsigned char)h->format;
    w.p += 4;
    put_nn(&w, (unsigned long long)h->numrecs);
    if (h->ndims == 0) {
        put_u32(&w, 0);
        put_nn(&w, 0);
    } else {
        put_u32(&w, CDF_DIMENSION);
        put_nn(&w, (unsigned long long)h->ndims);
        for (i = 0; i < h->ndims; i++) {
            put_name(&w, h->dims[i].name);
            put_nn(&w, (unsigned long long)h->dims[i].size);
        }
    }
    put_atts(&w, &h->gatts);
    if (h->nvars == 0) {
        put_u32(&w, 0);
        put_nn(&w, 0);
    } else {
        put_u32(&w, CDF_VARIABLE);
        put_nn(&w, (unsigned long long)h->nvars);
        for (i = 0; i < h->nvars; i++) {
            const cdf_var *v = &h->vars[i];
            put_name(&w, v->name);
            put_nn(&w, (unsigned long long)v->ndims);
            for (d = 0; d < v->ndims; d++) put_nn(&w, (unsigned long long)v->dimids[d]);
            put_atts(&w, &v->atts);
            put_u32(&w, (unsigned long long)v->xtype);
            if (h->format < 5)      /* vsize saturates at 2^32-1, ncmpio_header_put.c:347-360 */
                put_u32(&w, v->len > 4294967292LL ? 4294967295ULL : (unsigned long long)v->len);
            else
                put_u64(&w, (unsigned long long)v->len);
            if (h->format == 1) {
                if (v->begin > CDF_MAX_INT) return NC_EINTOVERFLOW;
                put_u32(&w, (unsigned long long)v->begin);
            } else {
                put_u64(&w, (unsigned long long)v->begin);
            }
        }
    }
    return (long long)(w.p - buf);
}

/* ------------------------------------------------------------------------ */
/* decoding                                                                 */
/* ------------------------------------------------------------------------ */
typedef struct rbuf {
    const unsigned char *b;
    size_t len, pos, limit;     /* bytes past the file end read as zero, up to limit */
    size_t file_size;
    int nn, format, strict;
} rbuf;

static int get_bytes(rbuf *r, void *out, size_t n)
{
    size_t have;
    if (r->pos + n > r->len && r->len < r->file_size) return CDF_NEED_MORE;  /* not read yet */
    if (r->pos + n > r->limit) return NC_ENOTNC;    /* header runs past the file */
    have = r->pos < r->len ? r->len - r->pos : 0;
    if (have > n) have = n;
    if (out != NULL) {
        if (have) memcpy(out, r->b + r->pos, have);
        if (have < n) memset((unsigned char *)out + have, 0, n - have);
    }
    r->pos += n;
    return NC_NOERR;
}

static int get_u32(rbuf *r, unsigned long long *v)
{
    unsigned char b[4];
    int err = get_bytes(r, b, 4);
    if (err) return err;
    *v = ((unsigned long long)b[0] << 24) | ((unsigned long long)b[1] << 16) | ((unsigned long long)b[2] << 8) | b[3];
    return NC_NOERR;
}

static int get_u64(rbuf *r, unsigned long long *v)
{
    unsigned long long hi, lo;
    int err = get_u32(r, &hi);
    if (!err) err = get_u32(r, &lo);
    if (!err) *v = (hi << 32) | lo;
    return err;
}

static int get_nn(rbuf *r, unsigned long long *v) { return r->nn == 8 ? get_u64(r, v) : get_u32(r, v); }

/* padding bytes: returns NC_ENULLPAD (non fatal) in strict mode when not null */
static int get_pad(rbuf *r, size_t pad)
{
    unsigned char p[4] = {0, 0, 0, 0};
    int err;
    if (pad == 0) return NC_NOERR;
    err = get_bytes(r, p, pad);
    if (err) return err;
    if (r->strict && (p[0] | p[1] | p[2])) return NC_ENULLPAD;
    return NC_NOERR;
}

static int get_name(rbuf *r, char **name)
{
    unsigned long long n;
    int err = get_nn(r, &n), perr;
    *name = NULL;
    if (err) return err;
    if (n > CDF_MAX_NAME) return NC_EMAXNAME;
    *name = (char *)malloc((size_t)n + 1);
    if (*name == NULL) return NC_ENOMEM;
    if ((err = get_bytes(r, *name, (size_t)n)) != NC_NOERR) { free(*name); *name = NULL; return err; }
    (*name)[n] = '\0';
    perr = get_pad(r, (size_t)(RNDUP((long long)n, 4) - (long long)n));
    if (perr == NC_ENULLPAD) return perr;
    if (perr) { free(*name); *name = NULL; }
    return perr;
}

static int get_type(rbuf *r, int *xtype)
{
    unsigned long long t;
    int err = get_u32(r, &t);
    if (err) return err;
    if (t < NC_BYTE) return NC_EBADTYPE;
    if (r->format < 5 ? t > NC_DOUBLE : t > NC_UINT64) return NC_EBADTYPE;
    *xtype = (int)t;
    return NC_NOERR;
}

#define KEEP_PAD(e, status) do { if ((e) == NC_ENULLPAD) (status) = NC_ENULLPAD; else if (e) return (e); } while (0)

static int get_atts(rbuf *r, cdf_atts *a)
{
    unsigned long long tag, n;
    int err, status = NC_NOERR, i;
    if ((err = get_u32(r, &tag)) != NC_NOERR) return err;
    if ((err = get_nn(r, &n)) != NC_NOERR) return err;
    if (n > CDF_MAX_INT) return NC_EMAXATTS;
    if (n == 0) return NC_NOERR;
    if (tag != CDF_ATTRIBUTE) return NC_ENOTNC;
    for (i = 0; i < (int)n; i++) {
        char *name;
        int xtype, xl;
        unsigned long long ne;
        long long nbytes, xsz;
        err = get_name(r, &name);
        KEEP_PAD(err, status);
        if ((err = get_type(r, &xtype)) != NC_NOERR) { free(name); return err; }
        if ((err = get_nn(r, &ne)) != NC_NOERR) { free(name); return err; }
        xl = xlen_of(xtype);
        if (ne > (unsigned long long)CDF_MAX_INT64 / 8 ||
            r->pos + (size_t)(ne * (unsigned long long)xl) > r->limit) { free(name); return NC_ENOTNC; }
        nbytes = (long long)ne * xl;
        xsz = RNDUP(nbytes, 4);
        if (a->n == a->cap) {
            const int cap = a->cap ? 2 * a->cap : 8;
            cdf_att *nv = (cdf_att *)realloc(a->v, sizeof(cdf_att) * (size_t)cap);
            if (nv == NULL) { free(name); return NC_ENOMEM; }
            a->v = nv;
            a->cap = cap;
        }
        a->v[a->n].name = name;
        a->v[a->n].xtype = xtype;
        a->v[a->n].nelems = (long long)ne;
        a->v[a->n].xsz = xsz;
        a->v[a->n].xvalue = (unsigned char *)calloc(1, (size_t)(xsz ? xsz : 1));
        if (a->v[a->n].xvalue == NULL) { free(name); return NC_ENOMEM; }
        a->n++;
        if ((err = get_bytes(r, a->v[a->n - 1].xvalue, (size_t)nbytes)) != NC_NOERR) return err;
        /* attribute value padding is copied as read (kept zero in memory) */
        err = get_pad(r, (size_t)(xsz - nbytes));
        KEEP_PAD(err, status);
        memset(a->v[a->n - 1].xvalue + nbytes, 0, (size_t)(xsz - nbytes));
    }
    return status;
}

static int get_dims(rbuf *r, cdf_hdr *h)
{
    unsigned long long tag, n, len;
    int err, status = NC_NOERR, i;
    if ((err = get_u32(r, &tag)) != NC_NOERR) return err;
    if ((err = get_nn(r, &n)) != NC_NOERR) return err;
    if (n > CDF_MAX_INT) return NC_EMAXDIMS;
    if (n == 0) return NC_NOERR;
    if (tag != CDF_DIMENSION) return NC_ENOTNC;
    for (i = 0; i < (int)n; i++) {
        char *name;
        err = get_name(r, &name);
        KEEP_PAD(err, status);
        if ((err = get_nn(r, &len)) != NC_NOERR) { free(name); return err; }
        if (h->unlimited_id != -1 && len == 0) { free(name); return NC_EUNLIMIT; }
        /* NON_NEG: a CDF-5 length >= 2^63 would be negative as MPI_Offset;
         * the reference has no check and overflows later (no fixture pins a
         * code), so it is rejected here as a bad dimension size */
        if (len > (unsigned long long)CDF_MAX_INT64) { free(name); return NC_EDIMSIZE; }
        err = cdf_add_dim(h, name, (long long)len);
        free(name);
        if (err) return err;
    }
    return status;
}

static int get_vars(rbuf *r, cdf_hdr *h)
{
    unsigned long long tag, n, v64;
    int err, status = NC_NOERR, i, d;
    if ((err = get_u32(r, &tag)) != NC_NOERR) return err;
    if ((err = get_nn(r, &n)) != NC_NOERR) return err;
    if (n > CDF_MAX_INT) return NC_EMAXVARS;
    if (n == 0) return NC_NOERR;
    if (tag != CDF_VARIABLE) return NC_ENOTNC;
    for (i = 0; i < (int)n; i++) {
        char *name;
        unsigned long long nd;
        cdf_var *v;
        err = get_name(r, &name);
        KEEP_PAD(err, status);
        if ((err = get_nn(r, &nd)) != NC_NOERR) { free(name); return err; }
        if (nd > CDF_MAX_INT) { free(name); return NC_EMAXDIMS; }
        if (r->pos + nd * (unsigned long long)r->nn > r->limit) { free(name); return NC_ENOTNC; }
        err = cdf_add_var(h, name, NC_BYTE, (int)nd, NULL);
        free(name);
        if (err) return err;
        v = &h->vars[h->nvars - 1];
        for (d = 0; d < (int)nd; d++) {
            if ((err = get_nn(r, &v64)) != NC_NOERR) return err;
            if (v64 >= (unsigned long long)h->ndims) return NC_EBADDIM;
            v->dimids[d] = (int)v64;
        }
        err = get_atts(r, &v->atts);
        KEEP_PAD(err, status);
        if ((err = get_type(r, &v->xtype)) != NC_NOERR) return err;
        v->xsz = xlen_of(v->xtype);
        if ((err = get_nn(r, &v64)) != NC_NOERR) return err;       /* vsize: recomputed */
        v->len = (long long)v64;
        if (h->format == 1) err = get_u32(r, &v64);
        else err = get_u64(r, &v64);
        if (err) return err;
        v->begin = (long long)v64;
    }
    return status;
}

/* compute_var_shape, ncmpio_header_get.c:34-97 */
static int compute_var_shape(cdf_hdr *h)
{
    int i, err, last_fix = -1;
    const cdf_var *first_var = NULL, *first_rec = NULL;
    if (h->nvars == 0) return NC_NOERR;
    h->begin_var = h->xsz;
    h->begin_rec = h->xsz;
    h->recsize = 0;
    for (i = 0; i < h->nvars; i++) {
        cdf_var *v = &h->vars[i];
        if ((err = cdf_var_shape(v, h)) != NC_NOERR) return err;
        if (cdf_is_recvar(v)) {
            if (first_rec == NULL) first_rec = v;
            h->recsize += v->len;
        } else {
            if (first_var == NULL) first_var = v;
            h->begin_rec = v->begin + v->len;
            last_fix = i;
        }
    }
    h->fix_end = last_fix >= 0 ? h->vars[last_fix].begin + h->vars[last_fix].len : h->begin_var;
    if (first_rec != NULL) {
        if (h->begin_rec > first_rec->begin) return NC_ENOTNC;
        h->begin_rec = first_rec->begin;
        if (h->recsize == first_rec->len) h->recsize = first_rec->dsizes[0] * first_rec->xsz;
    }
    h->begin_var = first_var != NULL ? first_var->begin : h->begin_rec;
    if (h->begin_var <= 0 || h->xsz > h->begin_var || h->begin_rec <= 0 || h->begin_var > h->begin_rec)
        return NC_ENOTNC;
    return NC_NOERR;
}

int cdf_hdr_decode(const unsigned char *buf, size_t len, size_t file_size, cdf_hdr *h, int strict_pad)
{
    rbuf r;
    int err, status = NC_NOERR, i;
    unsigned long long nrec;
    cdf_hdr_init(h, 0);
    if (len > file_size) len = file_size;
    r.b = buf;
    r.len = len;
    r.file_size = file_size;
    r.pos = 0;
    r.limit = file_size + CDF_HDR_CHUNK;
    r.strict = strict_pad;
    if (len < 4 || memcmp(buf, "CDF", 3) != 0) return NC_ENOTNC;
    if (buf[3] != 1 && buf[3] != 2 && buf[3] != 5) return NC_ENOTNC;
    h->format = buf[3];
    r.format = h->format;
    r.nn = h->format == 5 ? 8 : 4;
    r.pos = 4;
    if ((err = get_nn(&r, &nrec)) != NC_NOERR) goto fail;
    h->numrecs = (long long)nrec;
    err = get_dims(&r, h);
    if (err == NC_ENULLPAD) status = err; else if (err) goto fail;
    err = get_atts(&r, &h->gatts);
    if (err == NC_ENULLPAD) status = err; else if (err) goto fail;
    err = get_vars(&r, h);
    if (err == NC_ENULLPAD) status = err; else if (err) goto fail;
    h->xsz = cdf_hdr_len(h);
    if ((err = compute_var_shape(h)) != NC_NOERR) goto fail;
    h->num_rec_vars = 0;
    for (i = 0; i < h->nvars; i++) h->num_rec_vars += cdf_is_recvar(&h->vars[i]);
    if ((err = cdf_check_vlens(h)) != NC_NOERR) goto fail;
    if ((err = cdf_check_voffs(h)) != NC_NOERR) goto fail;
    if (h->nvars == 0) {           /* no variables: the data section starts at the header end */
        h->begin_var = h->begin_rec = h->xsz;
    }
    return status;
fail:
    cdf_hdr_free(h);
    return err;
}

/* ------------------------------------------------------------------------ */
/* shapes, sizes, offsets                                                   */
/* ------------------------------------------------------------------------ */
static int check_vlen(const cdf_var *v, long long vlen_max)
{
    long long prod = v->xsz;
    int i;
    for (i = cdf_is_recvar(v) ? 1 : 0; i < v->ndims; i++) {
        if (v->shape[i] > vlen_max / prod) return 0;
        prod *= v->shape[i];
    }
    return 1;
}

int cdf_var_shape(cdf_var *v, const cdf_hdr *h)
{
    long long product = 1;
    int i;
    if (v->ndims > 0) {
        for (i = 0; i < v->ndims; i++) {
            v->shape[i] = h->dims[v->dimids[i]].size;
            if (v->shape[i] == 0 && i != 0) return NC_EUNLIMPOS;
        }
        /* size check before the products, so they cannot overflow (same
         * result as the reference, which multiplies first, ncmpio_var.c:310-332) */
        if (!check_vlen(v, CDF_MAX_INT64 - 3)) return NC_EVARSIZE;
        if (v->ndims == 1) {
            if (v->shape[0] == 0) v->dsizes[0] = 1;
            else { v->dsizes[0] = v->shape[0]; product = v->shape[0]; }
        } else {
            v->dsizes[v->ndims - 1] = v->shape[v->ndims - 1];
            product = v->shape[v->ndims - 1];
            for (i = v->ndims - 2; i >= 0; i--) {
                if (v->shape[i] != 0) product *= v->shape[i];
                v->dsizes[i] = product;
            }
        }
    }
    if (!check_vlen(v, CDF_MAX_INT64 - 3)) return NC_EVARSIZE;
    v->len = product * v->xsz;
    if (v->len % 4) v->len += 4 - v->len % 4;
    return NC_NOERR;
}

int cdf_check_vlens(const cdf_hdr *h)
{
    long long vlen_max, large_fix = 0, large_rec = 0, nrec = 0;
    int i, last = 0;
    if (h->nvars == 0) return NC_NOERR;
    vlen_max = h->format >= 5 ? CDF_MAX_INT64 - 3 : h->format == 2 ? CDF_MAX_UINT - 3 : CDF_MAX_INT - 3;
    for (i = 0; i < h->nvars; i++) {
        const cdf_var *v = &h->vars[i];
        if (cdf_is_recvar(v)) { nrec++; continue; }
        last = 0;
        if (!check_vlen(v, vlen_max)) {
            if (h->format >= 5) return NC_EVARSIZE;
            large_fix++;
            last = 1;
        }
    }
    if (large_fix > 1) return NC_EVARSIZE;
    if (large_fix == 1 && last == 0) return NC_EVARSIZE;
    if (nrec == 0) return NC_NOERR;
    if (large_fix == 1) return NC_EVARSIZE;
    for (i = 0; i < h->nvars; i++) {
        const cdf_var *v = &h->vars[i];
        if (!cdf_is_recvar(v)) continue;
        last = 0;
        if (!check_vlen(v, vlen_max)) {
            if (h->format >= 5) return NC_EVARSIZE;
            large_rec++;
            last = 1;
        }
    }
    if (large_rec > 1) return NC_EVARSIZE;
    if (large_rec == 1 && last == 0) return NC_EVARSIZE;
    return NC_NOERR;
}

int cdf_check_voffs(const cdf_hdr *h)
{
    long long prev_off;
    int i;
    if (h->nvars == 0) return NC_NOERR;
    if (h->nvars > h->num_rec_vars) {
        prev_off = h->begin_var;
        for (i = 0; i < h->nvars; i++) {
            const cdf_var *v = &h->vars[i];
            if (cdf_is_recvar(v)) continue;
            if (v->begin < prev_off) return NC_ENOTNC;
            prev_off = v->begin + v->len;
        }
        if (h->begin_rec < prev_off) return NC_ENOTNC;
    }
    if (h->num_rec_vars == 0) return NC_NOERR;
    prev_off = h->begin_rec;
    for (i = 0; i < h->nvars; i++) {
        const cdf_var *v = &h->vars[i];
        if (!cdf_is_recvar(v)) continue;
        if (v->begin < prev_off) return NC_ENOTNC;
        prev_off = v->begin + v->len;
    }
    return NC_NOERR;
}

int cdf_begins(cdf_hdr *h, const cdf_hdr *old)
{
    long long end_var;
    int i, j, nfix;
    const cdf_var *last = NULL;
    h->xsz = cdf_hdr_len(h);
    h->num_rec_vars = 0;
    for (i = 0; i < h->nvars; i++) h->num_rec_vars += cdf_is_recvar(&h->vars[i]);
    nfix = h->nvars - h->num_rec_vars;
    if (h->nvars == 0) {
        h->begin_var = h->begin_var > h->xsz ? h->begin_var : h->xsz;
        h->begin_rec = h->begin_var;
        h->recsize = 0;
        h->numrecs = 0;
        return NC_NOERR;
    }
    {   /* alignment arguments of ncmpi__enddef; 0 selects the default */
        const long long va = h->v_align > 0 ? RNDUP(h->v_align, 4) : CDF_DEFAULT_V_ALIGN;
        const long long ra = h->r_align > 0 ? RNDUP(h->r_align, 4)
                                            : (nfix > 0 ? CDF_DEFAULT_R_ALIGN : CDF_DEFAULT_V_ALIGN);
        if (h->begin_var < h->xsz + h->h_minfree) h->begin_var = h->xsz + h->h_minfree;
        if (old != NULL && h->begin_var < old->begin_var) h->begin_var = old->begin_var;
        if (nfix > 0) h->begin_var = RNDUP(h->begin_var, va);
        end_var = h->begin_var;
        for (j = 0, i = 0; i < h->nvars; i++) {
            cdf_var *v = &h->vars[i];
            if (cdf_is_recvar(v)) continue;
            if (h->format == 1 && end_var > CDF_MAX_INT) return NC_EVARSIZE;
            v->begin = RNDUP(end_var, 4);
            if (old != NULL) {
                for (; j < old->nvars; j++)
                    if (!cdf_is_recvar(&old->vars[j])) break;
                if (j < old->nvars) {
                    if (v->begin < old->vars[j].begin) v->begin = old->vars[j].begin;
                    j++;
                }
            }
            end_var = v->begin + v->len;
        }
        h->fix_end = RNDUP(end_var, 4);
        h->begin_rec = nfix > 0 ? h->fix_end + h->v_minfree : h->fix_end;
        if (old != NULL && h->begin_rec < old->begin_rec) h->begin_rec = old->begin_rec;
        h->begin_rec = RNDUP(h->begin_rec, ra);
        if (nfix == 0) h->begin_var = h->begin_rec;
        end_var = h->begin_rec;
        h->recsize = 0;
        for (j = 0, i = 0; i < h->nvars; i++) {
            cdf_var *v = &h->vars[i];
            if (!cdf_is_recvar(v)) continue;
            if (h->format == 1 && end_var > CDF_MAX_INT) return NC_EVARSIZE;
            v->begin = end_var;
            if (old != NULL) {
                for (; j < old->nvars; j++)
                    if (cdf_is_recvar(&old->vars[j])) break;
                if (j < old->nvars) {
                    if (v->begin < old->vars[j].begin) v->begin = old->vars[j].begin;
                    j++;
                }
            }
            end_var += v->len;
            h->recsize += v->len;
            last = v;
        }
        /* exactly one record variable: records are packed, no 4-byte pad */
        if (last != NULL && h->recsize == last->len) h->recsize = last->dsizes[0] * last->xsz;
    }
    return NC_NOERR;
}

/* ------------------------------------------------------------------------ */
/* fill patterns                                                            */
/* ------------------------------------------------------------------------ */
int cdf_default_fill(int xtype, unsigned char out[8])
{
    /* ncmpio_fill.c:50-60: NC_FILL_* in external (big-endian) order */
    static const unsigned char f_byte[1] = {0x81}, f_char[1] = {0x00}, f_short[2] = {0x80, 0x01},
        f_int[4] = {0x80, 0x00, 0x00, 0x01}, f_float[4] = {0x7C, 0xF0, 0x00, 0x00},
        f_double[8] = {0x47, 0x9E, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00}, f_ubyte[1] = {0xFF},
        f_ushort[2] = {0xFF, 0xFF}, f_uint[4] = {0xFF, 0xFF, 0xFF, 0xFF},
        f_int64[8] = {0x80, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x02},
        f_uint64[8] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFE};
    const unsigned char *src;
    switch (xtype) {
    case NC_BYTE: src = f_byte; break;
    case NC_CHAR: src = f_char; break;
    case NC_SHORT: src = f_short; break;
    case NC_INT: src = f_int; break;
    case NC_FLOAT: src = f_float; break;
    case NC_DOUBLE: src = f_double; break;
    case NC_UBYTE: src = f_ubyte; break;
    case NC_USHORT: src = f_ushort; break;
    case NC_UINT: src = f_uint; break;
    case NC_INT64: src = f_int64; break;
    case NC_UINT64: src = f_uint64; break;
    default: return NC_EBADTYPE;
    }
    memset(out, 0, 8);
    memcpy(out, src, (size_t)xlen_of(xtype));
    return NC_NOERR;
}

int cdf_var_fill(const cdf_var *v, unsigned char out[8])
{
    const int i = cdf_find_att(&v->atts, "_FillValue");
    if (i < 0) return cdf_default_fill(v->xtype, out);
    memset(out, 0, 8);
    /* ncmpio_fill.c:104-117: the attribute must hold one value of the variable's type */
    if (v->atts.v[i].xtype != v->xtype || v->atts.v[i].nelems != 1) return NC_EBADTYPE;
    memcpy(out, v->atts.v[i].xvalue, (size_t)v->xsz);
    return NC_NOERR;
}
