/*
 * pncx_cdf.h -- in-memory model of a classic CDF-1/2/5 header (internal).
 *
 * Mirrors the NC / NC_dim / NC_attr / NC_var objects of the reference
 * (src/drivers/ncmpio/ncmpio_NC.h:212-331) with only the fields the header
 * codec, the variable layout (NC_begins, ncmpio_enddef.c:359-612) and the
 * data path need.  Header encode/decode: pncx_cdf.c.
 */
#ifndef PNCX_CDF_H
#define PNCX_CDF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CDF_DIMENSION  0x0A   /* list tags, ncmpio_NC.h:62-66 */
#define CDF_VARIABLE   0x0B
#define CDF_ATTRIBUTE  0x0C

#define CDF_MAX_INT    2147483647LL
#define CDF_MAX_UINT   4294967295LL
#define CDF_MAX_INT64  9223372036854775807LL
#define CDF_MAX_NAME   256
#define CDF_HDR_CHUNK  262144           /* PNC_HDR_READ_CHUNK_SIZE, ncmpio_NC.h:86 */
#define CDF_DEFAULT_V_ALIGN 512         /* ncmpio_NC.h:43-56 */
#define CDF_DEFAULT_R_ALIGN 4

typedef struct cdf_dim {
    char     *name;
    long long size;                     /* 0 = NC_UNLIMITED */
} cdf_dim;

typedef struct cdf_att {
    char          *name;
    int            xtype;
    long long      nelems;
    long long      xsz;                 /* nelems*xlen rounded up to 4 */
    unsigned char *xvalue;              /* external (big-endian) bytes, xsz long, zero padded */
} cdf_att;

typedef struct cdf_atts {
    int      n, cap;
    cdf_att *v;
} cdf_atts;

typedef struct cdf_var {
    char      *name;
    int        ndims;
    int       *dimids;
    long long *shape;                   /* shape[0] = 0 for record variables */
    long long *dsizes;                  /* right-to-left products, ncmpio_var.c:304-327 */
    cdf_atts   atts;
    int        xtype;
    int        xsz;                     /* external element size */
    long long  len;                     /* bytes of one record (record var) or of the whole var, 4-aligned */
    long long  begin;
    int        no_fill;
} cdf_var;

typedef struct cdf_hdr {
    int        format;                  /* 1, 2 or 5 */
    long long  numrecs;
    int        ndims, capd, unlimited_id;
    cdf_dim   *dims;
    cdf_atts   gatts;
    int        nvars, capv, num_rec_vars;
    cdf_var   *vars;
    /* layout (NC_begins) */
    long long  xsz;                     /* header bytes, unaligned */
    long long  begin_var, begin_rec, recsize, fix_end;
    long long  h_minfree, v_align, v_minfree, r_align;
} cdf_hdr;

void      cdf_hdr_init(cdf_hdr *h, int format);
void      cdf_hdr_free(cdf_hdr *h);
int       cdf_hdr_copy(cdf_hdr *dst, const cdf_hdr *src);
long long cdf_hdr_len(const cdf_hdr *h);
/* Encode into buf (at least cdf_hdr_len bytes).  Returns bytes written or a
 * negative NC error. */
long long cdf_hdr_encode(const cdf_hdr *h, unsigned char *buf);
/* Decode from buf[0..len), the first len bytes of a file of file_size
 * bytes.  Bytes past the end of the FILE read as zero (the reference's
 * chunked fetch zero-fills a short read), up to one chunk; when the decoder
 * needs bytes in [len, file_size) it returns CDF_NEED_MORE and the caller
 * reads more and retries.  strict_pad: report non-null header padding as
 * NC_ENULLPAD (ncvalidator).  On success the layout fields are recomputed
 * (compute_var_shape) and the header is validated (check_vlens,
 * check_voffs). */
#define CDF_NEED_MORE 1
int       cdf_hdr_decode(const unsigned char *buf, size_t len, size_t file_size, cdf_hdr *h, int strict_pad);

int       cdf_check_name(const char *name);
int       cdf_find_dim(const cdf_hdr *h, const char *name);
int       cdf_find_var(const cdf_hdr *h, const char *name);
int       cdf_find_att(const cdf_atts *a, const char *name);
int       cdf_add_dim(cdf_hdr *h, const char *name, long long size);
int       cdf_add_var(cdf_hdr *h, const char *name, int xtype, int ndims, const int *dimids);
/* set (create or replace) an attribute from external bytes */
int       cdf_set_att(cdf_atts *a, const char *name, int xtype, long long nelems, const void *xvalue);
int       cdf_del_att(cdf_atts *a, const char *name);
int       cdf_var_shape(cdf_var *v, const cdf_hdr *h);   /* ncmpio_NC_var_shape64 */
int       cdf_check_vlens(const cdf_hdr *h);             /* ncmpio_NC_check_vlens */
int       cdf_check_voffs(const cdf_hdr *h);             /* ncmpio_NC_check_voffs */
/* NC_begins: compute xsz, begin of every variable, begin_var/rec, recsize.
 * old (may be NULL) is the header before redef: begins never move backwards. */
int       cdf_begins(cdf_hdr *h, const cdf_hdr *old);
/* the big-endian default fill pattern of xtype (ncmpio_fill.c:50-60) */
int       cdf_default_fill(int xtype, unsigned char out[8]);
/* the variable's fill pattern: _FillValue attribute bytes or the default */
int       cdf_var_fill(const cdf_var *v, unsigned char out[8]);
static inline int cdf_is_recvar(const cdf_var *v) { return v->ndims > 0 && v->shape[0] == 0; }

#ifdef __cplusplus
}
#endif
#endif
