/*
 * pnc_driver.c -- the MI355X driver: a struct PNC_driver (include/
 * pncx_dispatch.h, src/include/dispatch.h:63-125) with the semantics of the
 * reference's ncmpio driver (src/drivers/ncmpio/ncmpio_driver.c:15-73) whose
 * put/get buffers are converted by the HIP kernels of libpncx.so:
 *
 *   put_var/get_var, iput/iget/bput_var,
 *   put/get/iput/iget/bput_varn          -> pncx_nc_* (pncx_nc.h): the buffer
 *                                           policy of ncmpio_getput.m4 /
 *                                           ncmpio_i_getput.m4 with the GPU
 *                                           swap/convert (pncx.h)
 *   flexible buftypes (MPI derived)       -> pncx_ncmpi_*_varm (pncx_mpi.h):
 *                                           typemap fused into the kernels
 *   wait/cancel                           -> pncx_nc_wait_all: one batched
 *                                           conversion per flush
 *
 * Parallel files.  One process per GPU shares a file over an MPI
 * communicator.  Every rank keeps its own copy of the header and makes the
 * same define-mode calls; rank 0 alone writes the header, numrecs and the
 * fills, and moves data at enddef (ncmpio_enddef.c:681, ncmpio_sync.c:
 * 39-101); the other ranks' handles are created with
 * pncx_nc_create_shared(writer = 0) after rank 0 has created the file.
 * numrecs is made consistent with MPI_Allreduce(MAX) after every collective
 * put of a record variable, and written when it grows (ncmpio_getput.m4:
 * 272-311), at collective waits (ncmpio_wait.c:603-672), at end_indep_data,
 * sync and close (ncmpio_file_misc.c:206-216).  Data goes from each rank straight to its own
 * byte ranges of the file (POSIX I/O); there is no MPI-IO and no intra-node
 * aggregation, and so no data-path collective.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "../../include/pncx_dispatch.h"
#include "../../include/pncx_nc.h"
#include "../../include/pncx_ncmpii.h"
#include "../../include/pncx_mpi.h"

typedef struct stage_t {       /* a flexible varn request staged through a packed copy */
    int reqid, get;
    void *tmp;                 /* packed elements (MPI_Pack order) */
    void *user;
    MPI_Offset bufcount;
    MPI_Datatype buftype;      /* duplicated; freed with the stage */
    pncx_dtype *dt;            /* device buffers: the committed buftype, tmp in HBM */
} stage_t;

typedef struct NCM {
    int ncid;                  /* pncx_nc handle */
    int pub;                   /* the dispatcher's ncid */
    MPI_Comm comm;             /* the dispatcher's communicator (not owned) */
    int rank, nprocs;
    int indef, indep, rdonly, created;
    char *path;
    MPI_Info info;
    stage_t *stages;
    int nstage, capstage;
} NCM;

/* ------------------------------------------------------------------------ */
/* helpers                                                                   */
/* ------------------------------------------------------------------------ */
static int min_err(NCM *m, int err)
{
    int e = err;
    if (m->nprocs > 1) MPI_Allreduce(&err, &e, 1, MPI_INT, MPI_MIN, m->comm);
    return e;
}

static int num_rec_vars(NCM *m, int *nrec, int *nfix)
{
    int nvars = 0, unlim = -1, i, err, ndims, dimids[1024];
    *nrec = *nfix = 0;
    if ((err = pncx_nc_inq(m->ncid, NULL, &nvars, NULL, &unlim)) != NC_NOERR) return err;
    for (i = 0; i < nvars; i++) {
        if ((err = pncx_nc_inq_var(m->ncid, i, NULL, NULL, &ndims, NULL, NULL)) != NC_NOERR) return err;
        if (ndims > 0 && ndims <= 1024 &&
            (err = pncx_nc_inq_var(m->ncid, i, NULL, NULL, NULL, dimids, NULL)) != NC_NOERR)
            return err;
        if (ndims > 0 && unlim >= 0 && dimids[0] == unlim) (*nrec)++;
        else (*nfix)++;
    }
    return NC_NOERR;
}

static MPI_Offset my_numrecs(NCM *m)
{
    int unlim = -1;
    MPI_Offset n = 0;
    if (pncx_nc_inq(m->ncid, NULL, NULL, NULL, &unlim) == NC_NOERR && unlim >= 0)
        pncx_nc_inq_dim(m->ncid, unlim, NULL, &n);
    return n;
}

/* numrecs: the MAX over ranks in every rank's memory (ncmpio_sync_numrecs) */
static int sync_numrecs_mem(NCM *m)
{
    MPI_Offset n, mx;
    int unlim = -1;
    if (m->nprocs == 1) return NC_NOERR;
    /* every rank holds the same header, so all agree whether to reduce */
    if (pncx_nc_inq(m->ncid, NULL, NULL, NULL, &unlim) != NC_NOERR || unlim < 0) return NC_NOERR;
    n = my_numrecs(m);
    if (MPI_Allreduce(&n, &mx, 1, MPI_OFFSET, MPI_MAX, m->comm) != MPI_SUCCESS) return NC_EMPI;
    return pncx_nc_set_numrecs(m->ncid, mx);
}

static void barrier(NCM *m)
{
    if (m->nprocs > 1) MPI_Barrier(m->comm);
}

/* the variable's own native itype (MPI_DATATYPE_NULL buftype, dtype_decode.c:657-668) */
static int native_itype(NCM *m, int varid)
{
    int xtype = 0;
    if (pncx_nc_inq_var(m->ncid, varid, NULL, &xtype, NULL, NULL, NULL) != NC_NOERR) return 0;
    switch (xtype) {
    case NC_BYTE: return PNCX_ITYPE_SCHAR;
    case NC_CHAR: return PNCX_ITYPE_CHAR;
    case NC_SHORT: return PNCX_ITYPE_SHORT;
    case NC_INT: return PNCX_ITYPE_INT;
    case NC_FLOAT: return PNCX_ITYPE_FLOAT;
    case NC_DOUBLE: return PNCX_ITYPE_DOUBLE;
    case NC_UBYTE: return PNCX_ITYPE_UCHAR;
    case NC_USHORT: return PNCX_ITYPE_USHORT;
    case NC_UINT: return PNCX_ITYPE_UINT;
    case NC_INT64: return PNCX_ITYPE_LONGLONG;
    case NC_UINT64: return PNCX_ITYPE_ULONGLONG;
    default: return 0;
    }
}

/* a buffer description that needs no packing: the high-level form
 * (bufcount -1), MPI_DATATYPE_NULL, or a predefined buftype */
static int direct_itype(NCM *m, int varid, MPI_Offset bufcount, MPI_Datatype buftype, int *itype)
{
    if (buftype == MPI_DATATYPE_NULL) { *itype = native_itype(m, varid); return 1; }
    *itype = pncx_itype_from_mpi(buftype);
    if (bufcount == -1) return 1;
    return *itype != 0;
}

static MPI_Offset varn_nelems(NCM *m, int varid, int num, MPI_Offset *const *counts)
{
    int ndims = 0, i, d;
    MPI_Offset total = 0;
    pncx_nc_inq_var(m->ncid, varid, NULL, NULL, &ndims, NULL, NULL);
    for (i = 0; i < num; i++) {
        MPI_Offset n = 1;
        if (counts != NULL && counts[i] != NULL)
            for (d = 0; d < ndims; d++) n *= counts[i][d];
        total += n;
    }
    return total;
}

/* A flexible varn with a derived buftype: the reference packs it with
 * MPI_Pack before the conversion (ncmpio_i_varn.m4:165-231 ->
 * ncmpio_pack_xbuf); here the packed copy becomes a contiguous buffer of
 * the buftype's element type for the GPU conversion. */
static int pack_flex(const void *buf, MPI_Offset bufcount, MPI_Datatype buftype, MPI_Offset want, int pack,
                     void **tmp, int *itype)
{
    MPI_Offset nblk, ext, *disp = NULL, *blen = NULL, per = 0, i;
    int err, tsize, pos = 0, esize;
    *tmp = NULL;
    err = pncx_mpi_type_flatten(buftype, itype, &nblk, &disp, &blen, &ext);
    if (err) return err;
    for (i = 0; i < nblk; i++) per += blen[i];
    free(disp);
    free(blen);
    if (bufcount < 0 || per * bufcount != want) return NC_EIOMISMATCH;
    if (MPI_Type_size(buftype, &tsize) != MPI_SUCCESS) return NC_EMPI;
    esize = pncx_ilen(*itype);
    if (esize <= 0 || (MPI_Offset)tsize != per * esize) return NC_EBADTYPE;
    *tmp = malloc((size_t)(want * esize) + 1);
    if (*tmp == NULL) return NC_ENOMEM;
    if (pack && want > 0 &&
        MPI_Pack(buf, (int)bufcount, buftype, *tmp, (int)(want * esize), &pos, MPI_COMM_SELF) != MPI_SUCCESS) {
        free(*tmp);
        *tmp = NULL;
        return NC_EMPI;
    }
    return NC_NOERR;
}

static int unpack_flex(const void *tmp, MPI_Offset want, int itype, void *buf, MPI_Offset bufcount,
                       MPI_Datatype buftype)
{
    int pos = 0;
    if (want == 0) return NC_NOERR;
    if (MPI_Unpack(tmp, (int)(want * pncx_ilen(itype)), &pos, buf, (int)bufcount, buftype, MPI_COMM_SELF) !=
        MPI_SUCCESS)
        return NC_EMPI;
    return NC_NOERR;
}

/* a packed copy in HBM for a derived buftype over a device buffer: the
 * MPI library here is not GPU-aware, so the pack is pncx_dev_pack (the
 * typemap kernels) instead of MPI_Pack */
static int pack_flex_dev(const void *buf, MPI_Offset bufcount, MPI_Datatype buftype, MPI_Offset want, int pack,
                         void **tmp, int *itype, pncx_dtype **dt)
{
    pncx_offset tn = 0;
    int err;
    *tmp = NULL;
    *dt = NULL;
    if ((err = pncx_mpi_type_commit(buftype, dt)) != NC_NOERR) return err;
    pncx_type_inq(*dt, itype, &tn, NULL, NULL);
    if (bufcount < 0 || tn * bufcount != want) err = NC_EIOMISMATCH;
    if (!err && (*tmp = pncx_dev_alloc(want * pncx_ilen(*itype) + 16)) == NULL) err = PNCX_EDEVICE;
    if (!err && pack) err = pncx_dev_pack(*tmp, buf, bufcount, *dt, NULL);
    if (err) {
        pncx_dev_free(*tmp);
        pncx_type_free(*dt);
        *tmp = NULL;
        *dt = NULL;
    }
    return err;
}

static void free_packed(void *tmp, pncx_dtype *dt)
{
    if (dt != NULL) {
        pncx_dev_free(tmp);
        pncx_type_free(dt);
    } else {
        free(tmp);
    }
}

static int add_stage(NCM *m, int reqid, int get, void *tmp, void *user, MPI_Offset bufcount,
                     MPI_Datatype buftype, pncx_dtype *dt)
{
    stage_t *s;
    if (m->nstage == m->capstage) {
        const int cap = m->capstage ? 2 * m->capstage : 16;
        stage_t *ns = (stage_t *)realloc(m->stages, sizeof(stage_t) * (size_t)cap);
        if (ns == NULL) return NC_ENOMEM;
        m->stages = ns;
        m->capstage = cap;
    }
    s = &m->stages[m->nstage];
    s->reqid = reqid;
    s->get = get;
    s->tmp = tmp;
    s->user = user;
    s->bufcount = bufcount;
    s->dt = dt;
    if (MPI_Type_dup(buftype, &s->buftype) != MPI_SUCCESS) return NC_EMPI;
    m->nstage++;
    return NC_NOERR;
}

/* requests done (waited or cancelled): unpack staged gets, free the stages */
static int finish_stages(NCM *m, int nreqs, const int *ids, int unpack)
{
    int i, k, err = NC_NOERR;
    for (i = 0; i < m->nstage;) {
        stage_t *s = &m->stages[i];
        int hit = nreqs == NC_REQ_ALL || (nreqs == NC_PUT_REQ_ALL && !s->get) ||
                  (nreqs == NC_GET_REQ_ALL && s->get);
        for (k = 0; k < nreqs && !hit; k++) hit = ids[k] == s->reqid;
        if (!hit) { i++; continue; }
        if (unpack && s->get && s->dt != NULL) {
            const int e2 = pncx_dev_unpack(s->tmp, s->user, s->bufcount, s->dt, NULL);
            if (err == NC_NOERR) err = e2;
        } else if (unpack && s->get) {
            int itype;
            MPI_Offset nblk, ext, *disp = NULL, *blen = NULL, per = 0, j;
            if (pncx_mpi_type_flatten(s->buftype, &itype, &nblk, &disp, &blen, &ext) == NC_NOERR) {
                for (j = 0; j < nblk; j++) per += blen[j];
                free(disp);
                free(blen);
                if (err == NC_NOERR) err = unpack_flex(s->tmp, per * s->bufcount, itype, s->user, s->bufcount,
                                                       s->buftype);
            }
        }
        free_packed(s->tmp, s->dt);
        MPI_Type_free(&s->buftype);
        m->stages[i] = m->stages[--m->nstage];
    }
    return err;
}

/* ------------------------------------------------------------------------ */
/* files                                                                     */
/* ------------------------------------------------------------------------ */
static NCM *new_ncm(MPI_Comm comm, const char *path, int pub, MPI_Info info)
{
    NCM *m = (NCM *)calloc(1, sizeof *m);
    if (m == NULL) return NULL;
    m->ncid = -1;              /* pncx_nc ids start at 0: -1 = no handle yet */
    m->comm = comm;
    m->pub = pub;
    MPI_Comm_rank(comm, &m->rank);
    MPI_Comm_size(comm, &m->nprocs);
    m->path = strdup(path);
    m->info = MPI_INFO_NULL;
    if (info != MPI_INFO_NULL) MPI_Info_dup(info, &m->info);
    if (m->path == NULL) { free(m); return NULL; }
    return m;
}

static void free_ncm(NCM *m)
{
    if (m == NULL) return;
    finish_stages(m, NC_REQ_ALL, NULL, 0);
    free(m->stages);
    if (m->info != MPI_INFO_NULL) MPI_Info_free(&m->info);
    free(m->path);
    free(m);
}

static int drv_create(MPI_Comm comm, const char *path, int cmode, int ncid, int env_mode, MPI_Info info,
                      PNC_comm_attr attr, void **ncpp)
{
    NCM *m;
    int err = NC_NOERR, root_err = NC_NOERR;
    (void)env_mode;
    (void)attr;
    m = new_ncm(comm, path, ncid, info);
    if (m == NULL) return NC_ENOMEM;
    /* rank 0 creates (and truncates) the file, then the others open it */
    if (m->rank == 0) root_err = err = pncx_nc_create(path, cmode, &m->ncid);
    if (m->nprocs > 1) MPI_Bcast(&root_err, 1, MPI_INT, 0, comm);
    if (root_err != NC_NOERR) { free_ncm(m); return root_err; }
    if (m->rank > 0) err = pncx_nc_create_shared(path, cmode, 0, &m->ncid);
    if ((err = min_err(m, err)) != NC_NOERR) {
        /* the create failed on some rank: every rank drops its handle
         * without writing (no header, no numrecs) and rank 0 removes the
         * file it created, as ncmpio_abort does for a file still in its
         * first define mode; a rank whose own create failed has no handle
         * (m->ncid < 0) and must not close the unrelated file holding id 0 */
        if (m->ncid >= 0) {
            pncx_nc_set_writer(m->ncid, 0);
            pncx_nc_close(m->ncid);
        }
        barrier(m);
        if (m->rank == 0) unlink(path);
        free_ncm(m);
        return err;
    }
    m->indef = 1;
    m->created = 1;
    *ncpp = m;
    return NC_NOERR;
}

static int drv_open(MPI_Comm comm, const char *path, int omode, int ncid, int env_mode, MPI_Info info,
                    PNC_comm_attr attr, void **ncpp)
{
    NCM *m;
    int err;
    (void)env_mode;
    (void)attr;
    m = new_ncm(comm, path, ncid, info);
    if (m == NULL) return NC_ENOMEM;
    err = pncx_nc_open(path, omode, &m->ncid);
    if (err == NC_NOERR && m->rank > 0) err = pncx_nc_set_writer(m->ncid, 0);
    if ((err = min_err(m, err)) != NC_NOERR) {
        if (m->ncid >= 0) {              /* opened here, failed elsewhere: drop it unwritten */
            pncx_nc_set_writer(m->ncid, 0);
            pncx_nc_close(m->ncid);
        }
        free_ncm(m);
        return err;
    }
    m->rdonly = !(omode & NC_WRITE);
    *ncpp = m;
    return NC_NOERR;
}

static int drv_close(void *ncp)
{
    NCM *m = (NCM *)ncp;
    int err = NC_NOERR, e2;
    if (m->indef) {               /* close in define mode ends it first (ncmpio_close.c:72-80) */
        err = pncx_nc_enddef(m->ncid);
        barrier(m);
        m->indef = 0;
    }
    if (!m->rdonly) sync_numrecs_mem(m);
    e2 = pncx_nc_close(m->ncid);              /* rank 0 writes numrecs */
    if (err == NC_NOERR) err = e2;
    finish_stages(m, NC_REQ_ALL, NULL, 0);
    barrier(m);
    free_ncm(m);
    return err;
}

static int drv_enddef(void *ncp)
{
    NCM *m = (NCM *)ncp;
    int err = pncx_nc_enddef(m->ncid);       /* rank 0 writes the header, moves data, fills */
    barrier(m);                               /* no rank writes data before the fills are done */
    err = min_err(m, err);
    if (err == NC_NOERR) m->indef = 0;
    m->indep = 0;
    return err;
}

static int drv__enddef(void *ncp, MPI_Offset h_minfree, MPI_Offset v_align, MPI_Offset v_minfree,
                       MPI_Offset r_align)
{
    NCM *m = (NCM *)ncp;
    int err = pncx_nc__enddef(m->ncid, h_minfree, v_align, v_minfree, r_align);
    barrier(m);
    err = min_err(m, err);
    if (err == NC_NOERR) m->indef = 0;
    m->indep = 0;
    return err;
}

static int drv_redef(void *ncp)
{
    NCM *m = (NCM *)ncp;
    int err;
    sync_numrecs_mem(m);                      /* redef leaves independent mode too */
    m->indep = 0;
    err = pncx_nc_redef(m->ncid);
    if (err == NC_NOERR) m->indef = 1;
    return err;
}

static int drv_sync(void *ncp)
{
    NCM *m = (NCM *)ncp;
    int err;
    if (m->indef) return NC_EINDEFINE;
    sync_numrecs_mem(m);
    err = pncx_nc_sync(m->ncid);
    barrier(m);
    return err;
}

static int drv_flush(void *ncp)
{
    NCM *m = (NCM *)ncp;
    if (m->indef) return NC_EINDEFINE;
    return pncx_nc_sync(m->ncid);             /* POSIX I/O has no write-behind buffer to flush */
}

static int drv_abort(void *ncp)
{
    NCM *m = (NCM *)ncp;
    /* a file still in its first define mode is removed (ncmpio_abort) */
    const int unlink_it = m->created && m->indef;
    int err;
    if (unlink_it) {
        pncx_nc_set_writer(m->ncid, 0);          /* write nothing */
        err = pncx_nc_close(m->ncid);
        barrier(m);
        if (m->rank == 0) unlink(m->path);
    } else {
        if (m->indef) pncx_nc_set_writer(m->ncid, 0);   /* discard the redef */
        err = pncx_nc_close(m->ncid);
        barrier(m);
    }
    free_ncm(m);
    return err;
}

static int drv_set_fill(void *ncp, int fillmode, int *old)
{
    return pncx_nc_set_fill(((NCM *)ncp)->ncid, fillmode, old);
}

static int drv_inq(void *ncp, int *ndims, int *nvars, int *ngatts, int *unlimdimid)
{
    return pncx_nc_inq(((NCM *)ncp)->ncid, ndims, nvars, ngatts, unlimdimid);
}

static int drv_inq_misc(void *ncp, int *pathlen, char *path, int *num_fix_varsp, int *num_rec_varsp,
                        int *striping_size, int *striping_count, MPI_Offset *header_size,
                        MPI_Offset *header_extent, MPI_Offset *recsize, MPI_Offset *put_size,
                        MPI_Offset *get_size, MPI_Info *info_used, int *nreqs, MPI_Offset *usage,
                        MPI_Offset *buf_size)
{
    NCM *m = (NCM *)ncp;
    int err = NC_NOERR;
    if (pathlen) *pathlen = (int)strlen(m->path);
    if (path) strcpy(path, m->path);
    if (num_fix_varsp || num_rec_varsp) {
        int nrec, nfix;
        if ((err = num_rec_vars(m, &nrec, &nfix)) != NC_NOERR) return err;
        if (num_fix_varsp) *num_fix_varsp = nfix;
        if (num_rec_varsp) *num_rec_varsp = nrec;
    }
    if (striping_size) *striping_size = 0;      /* not a striped file system */
    if (striping_count) *striping_count = 0;
    if (header_size && (err = pncx_nc_inq_header_size(m->ncid, header_size)) != NC_NOERR) return err;
    if (header_extent && (err = pncx_nc_inq_header_extent(m->ncid, header_extent)) != NC_NOERR) return err;
    if (recsize && (err = pncx_nc_inq_recsize(m->ncid, recsize)) != NC_NOERR) return err;
    if (put_size || get_size) {
        MPI_Offset p = 0, g = 0;
        if ((err = pncx_nc_inq_io_size(m->ncid, &p, &g)) != NC_NOERR) return err;
        if (put_size) *put_size = p;
        if (get_size) *get_size = g;
    }
    if (info_used) {                            /* the hints this driver honours */
        char v[32];
        if (m->info != MPI_INFO_NULL) MPI_Info_dup(m->info, info_used);
        else MPI_Info_create(info_used);
        MPI_Info_set(*info_used, "pnetcdf_driver", "mi355x");
        MPI_Info_set(*info_used, "nc_in_place_swap", "disable");
        snprintf(v, sizeof v, "%d", 512);
        MPI_Info_set(*info_used, "nc_var_align_size", v);
    }
    if (nreqs && (err = pncx_nc_inq_nreqs(m->ncid, nreqs)) != NC_NOERR) return err;
    if (usage && (err = pncx_nc_inq_buffer_usage(m->ncid, usage)) != NC_NOERR) return err;
    if (buf_size && (err = pncx_nc_inq_buffer_size(m->ncid, buf_size)) != NC_NOERR) return err;
    return NC_NOERR;
}

static int drv_sync_numrecs(void *ncp)
{
    NCM *m = (NCM *)ncp;
    int err;
    if (m->indef) return NC_EINDEFINE;
    sync_numrecs_mem(m);
    err = m->rdonly ? NC_NOERR : pncx_nc_sync_numrecs(m->ncid, my_numrecs(m));
    barrier(m);
    return err;
}

static int drv_begin_indep_data(void *ncp)
{
    NCM *m = (NCM *)ncp;
    if (m->indef) return NC_EINDEFINE;
    if (m->indep) return NC_NOERR;            /* not an error since 1.2.0 */
    m->indep = 1;
    barrier(m);
    return NC_NOERR;
}

static int drv_end_indep_data(void *ncp)
{
    NCM *m = (NCM *)ncp;
    int err = NC_NOERR;
    if (m->indef) return NC_EINDEFINE;
    if (!m->indep) return NC_NOERR;           /* not an error since 1.9.0 */
    if (!m->rdonly) {
        sync_numrecs_mem(m);
        err = pncx_nc_sync_numrecs(m->ncid, my_numrecs(m));
    }
    m->indep = 0;
    return err;
}

/* ------------------------------------------------------------------------ */
/* dimensions, attributes, variables                                         */
/* ------------------------------------------------------------------------ */
static int drv_def_dim(void *ncp, const char *name, MPI_Offset len, int *dimid)
{
    return pncx_nc_def_dim(((NCM *)ncp)->ncid, name, len, dimid);
}

static int drv_inq_dimid(void *ncp, const char *name, int *dimid)
{
    return pncx_nc_inq_dimid(((NCM *)ncp)->ncid, name, dimid);
}

static int drv_inq_dim(void *ncp, int dimid, char *name, MPI_Offset *len)
{
    return pncx_nc_inq_dim(((NCM *)ncp)->ncid, dimid, name, len);
}

static int drv_rename_dim(void *ncp, int dimid, const char *name)
{
    return pncx_nc_rename_dim(((NCM *)ncp)->ncid, dimid, name);
}

static int drv_inq_att(void *ncp, int varid, const char *name, nc_type *xtype, MPI_Offset *len)
{
    return pncx_nc_inq_att(((NCM *)ncp)->ncid, varid, name, xtype, len);
}

static int drv_inq_attid(void *ncp, int varid, const char *name, int *idp)
{
    NCM *m = (NCM *)ncp;
    char nm[NC_MAX_NAME + 1];
    int natts = 0, i, err;
    err = varid == NC_GLOBAL ? pncx_nc_inq(m->ncid, NULL, NULL, &natts, NULL)
                             : pncx_nc_inq_var(m->ncid, varid, NULL, NULL, NULL, NULL, &natts);
    if (err) return err;
    for (i = 0; i < natts; i++) {
        if ((err = pncx_nc_inq_attname(m->ncid, varid, i, nm)) != NC_NOERR) return err;
        if (strcmp(nm, name) == 0) {
            if (idp) *idp = i;
            return NC_NOERR;
        }
    }
    return NC_ENOTATT;
}

static int drv_inq_attname(void *ncp, int varid, int attnum, char *name)
{
    return pncx_nc_inq_attname(((NCM *)ncp)->ncid, varid, attnum, name);
}

static int xtype_itype(int xtype)
{
    switch (xtype) {
    case NC_CHAR: return PNCX_ITYPE_CHAR;
    case NC_BYTE: return PNCX_ITYPE_SCHAR;
    case NC_UBYTE: return PNCX_ITYPE_UCHAR;
    case NC_SHORT: return PNCX_ITYPE_SHORT;
    case NC_USHORT: return PNCX_ITYPE_USHORT;
    case NC_INT: return PNCX_ITYPE_INT;
    case NC_UINT: return PNCX_ITYPE_UINT;
    case NC_FLOAT: return PNCX_ITYPE_FLOAT;
    case NC_DOUBLE: return PNCX_ITYPE_DOUBLE;
    case NC_INT64: return PNCX_ITYPE_LONGLONG;
    case NC_UINT64: return PNCX_ITYPE_ULONGLONG;
    default: return 0;
    }
}

/* ncmpio_copy_att: read in the attribute's own type, write it unchanged */
static int drv_copy_att(void *ncp_in, int varid_in, const char *name, void *ncp_out, int varid_out)
{
    NCM *mi = (NCM *)ncp_in, *mo = (NCM *)ncp_out;
    nc_type xtype;
    MPI_Offset len;
    int err, it;
    void *b;
    if ((err = pncx_nc_inq_att(mi->ncid, varid_in, name, &xtype, &len)) != NC_NOERR) return err;
    it = xtype_itype(xtype);
    b = malloc((size_t)(len > 0 ? len : 1) * 8);
    if (b == NULL) return NC_ENOMEM;
    err = pncx_nc_get_att(mi->ncid, varid_in, name, b, it);
    if (err == NC_NOERR) err = pncx_nc_put_att(mo->ncid, varid_out, name, xtype, len, b, it);
    free(b);
    return err;
}

static int drv_rename_att(void *ncp, int varid, const char *name, const char *newname)
{
    return pncx_nc_rename_att(((NCM *)ncp)->ncid, varid, name, newname);
}

static int drv_del_att(void *ncp, int varid, const char *name)
{
    return pncx_nc_del_att(((NCM *)ncp)->ncid, varid, name);
}

static int drv_get_att(void *ncp, int varid, const char *name, void *buf, MPI_Datatype itype)
{
    const int it = pncx_itype_from_mpi(itype);
    if (it == 0) return NC_EBADTYPE;
    return pncx_nc_get_att(((NCM *)ncp)->ncid, varid, name, buf, it);
}

static int drv_put_att(void *ncp, int varid, const char *name, nc_type xtype, MPI_Offset nelems,
                       const void *buf, MPI_Datatype itype)
{
    const int it = pncx_itype_from_mpi(itype);
    if (it == 0) return NC_EBADTYPE;
    return pncx_nc_put_att(((NCM *)ncp)->ncid, varid, name, xtype, nelems, buf, it);
}

static int drv_def_var(void *ncp, const char *name, nc_type xtype, int ndims, const int *dimids, int *varid)
{
    return pncx_nc_def_var(((NCM *)ncp)->ncid, name, xtype, ndims, dimids, varid);
}

static int drv_def_var_fill(void *ncp, int varid, int no_fill, const void *fill_value)
{
    return pncx_nc_def_var_fill(((NCM *)ncp)->ncid, varid, no_fill, fill_value);
}

static int drv_fill_var_rec(void *ncp, int varid, MPI_Offset recno)
{
    NCM *m = (NCM *)ncp;
    int err = NC_NOERR;
    /* collective (ncmpio_fill.c): every rank checks, rank 0 writes */
    if (m->rank == 0 || m->nprocs == 1) err = pncx_nc_fill_var_rec(m->ncid, varid, recno);
    if (m->nprocs > 1) {
        MPI_Bcast(&err, 1, MPI_INT, 0, m->comm);
        if (err == NC_NOERR && m->rank > 0) {
            MPI_Offset n = my_numrecs(m);
            if (recno + 1 > n) pncx_nc_set_numrecs(m->ncid, recno + 1);
        }
    }
    return err;
}

static int drv_inq_var(void *ncp, int varid, char *name, nc_type *xtype, int *ndims, int *dimids, int *natts,
                       MPI_Offset *offset, int *no_fill, void *fill_value)
{
    NCM *m = (NCM *)ncp;
    int err = NC_NOERR;
    if (varid == NC_GLOBAL) return pncx_nc_inq(m->ncid, NULL, NULL, natts, NULL);
    if (name || xtype || ndims || dimids || natts)
        err = pncx_nc_inq_var(m->ncid, varid, name, xtype, ndims, dimids, natts);
    if (!err && offset) err = pncx_nc_inq_varoffset(m->ncid, varid, offset);
    if (!err && (no_fill || fill_value)) err = pncx_nc_inq_var_fill(m->ncid, varid, no_fill, fill_value);
    return err;
}

static int drv_inq_varid(void *ncp, const char *name, int *varid)
{
    return pncx_nc_inq_varid(((NCM *)ncp)->ncid, name, varid);
}

static int drv_rename_var(void *ncp, int varid, const char *name)
{
    return pncx_nc_rename_var(((NCM *)ncp)->ncid, varid, name);
}

/* ------------------------------------------------------------------------ */
/* data                                                                      */
/* ------------------------------------------------------------------------ */
/* does varid run along the unlimited dimension (IS_RECVAR) */
static int is_recvar(NCM *m, int varid)
{
    int unlim = -1, ndims = 0, *dimids, rec;
    if (pncx_nc_inq(m->ncid, NULL, NULL, NULL, &unlim) != NC_NOERR || unlim < 0) return 0;
    if (pncx_nc_inq_var(m->ncid, varid, NULL, NULL, &ndims, NULL, NULL) != NC_NOERR || ndims <= 0) return 0;
    dimids = (int *)malloc(sizeof(int) * (size_t)ndims);
    if (dimids == NULL) return 0;
    rec = pncx_nc_inq_var(m->ncid, varid, NULL, NULL, NULL, dimids, NULL) == NC_NOERR && dimids[0] == unlim;
    free(dimids);
    return rec;
}

/* After a collective put of a record variable (ncmpio_getput.m4:272-311):
 * the MAX of every rank's record count, and if that grew past the count
 * all ranks agreed on before the put, the new value is written to the file
 * now (ncmpio_write_numrecs, :307; rank 0 is the writer).  Fixed-size
 * variables and independent puts touch nothing here (independent puts
 * are synced at the next collective call, :312-320). */
static int coll_put_done(NCM *m, int varid, int reqMode, MPI_Offset before)
{
    MPI_Offset n, mx;
    if (!(reqMode & NC_REQ_COLL) || !(reqMode & NC_REQ_WR) || !is_recvar(m, varid)) return NC_NOERR;
    n = mx = my_numrecs(m);
    if (m->nprocs > 1 && MPI_Allreduce(&n, &mx, 1, MPI_OFFSET, MPI_MAX, m->comm) != MPI_SUCCESS) return NC_EMPI;
    if (before < mx) return pncx_nc_sync_numrecs(m->ncid, mx);
    return NC_NOERR;
}

static int drv_put_var(void *ncp, int varid, const MPI_Offset *start, const MPI_Offset *count,
                       const MPI_Offset *stride, const MPI_Offset *imap, const void *buf, MPI_Offset bufcount,
                       MPI_Datatype buftype, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int err = NC_NOERR, it, e2;
    const MPI_Offset before = my_numrecs(m);
    if (!(reqMode & NC_REQ_ZERO)) {
        if (direct_itype(m, varid, bufcount, buftype, &it) && (bufcount == -1 || buftype == MPI_DATATYPE_NULL))
            err = pncx_nc_put_varm(m->ncid, varid, start, count, stride, imap, buf, it);
        else
            err = pncx_ncmpi_put_varm(m->ncid, varid, start, count, stride, imap, buf, bufcount, buftype);
    }
    e2 = coll_put_done(m, varid, reqMode, before);
    return (err == NC_NOERR || err == NC_ERANGE) && e2 != NC_NOERR ? e2 : err;
}

static int drv_get_var(void *ncp, int varid, const MPI_Offset *start, const MPI_Offset *count,
                       const MPI_Offset *stride, const MPI_Offset *imap, void *buf, MPI_Offset bufcount,
                       MPI_Datatype buftype, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int it;
    if (reqMode & NC_REQ_ZERO) return NC_NOERR;
    if (direct_itype(m, varid, bufcount, buftype, &it) && (bufcount == -1 || buftype == MPI_DATATYPE_NULL))
        return pncx_nc_get_varm(m->ncid, varid, start, count, stride, imap, buf, it);
    return pncx_ncmpi_get_varm(m->ncid, varid, start, count, stride, imap, buf, bufcount, buftype);
}

/* a varn buffer as (contiguous pointer, itype): predefined types directly,
 * derived buftypes through a packed copy */
static int varn_buffer(NCM *m, int varid, int num, MPI_Offset *const *counts, const void *buf,
                       MPI_Offset bufcount, MPI_Datatype buftype, int pack, void **tmp, const void **ptr, int *itype,
                       pncx_dtype **dt)
{
    MPI_Offset want = varn_nelems(m, varid, num, counts);
    *tmp = NULL;
    *ptr = buf;
    *dt = NULL;
    if (direct_itype(m, varid, bufcount, buftype, itype)) {
        if (*itype == 0) return NC_EBADTYPE;
        if (bufcount != -1 && buftype != MPI_DATATYPE_NULL && bufcount != want) return NC_EIOMISMATCH;
        return NC_NOERR;
    }
    /* a derived buftype over a buffer in HBM: packed on the device */
    if (pncx_is_device_ptr(buf)) {
        int err = pack_flex_dev(buf, bufcount, buftype, want, pack, tmp, itype, dt);
        if (err) return err;
        *ptr = *tmp;
        return NC_NOERR;
    }
    {
        int err = pack_flex(buf, bufcount, buftype, want, pack, tmp, itype);
        if (err) return err;
        *ptr = *tmp;
        return NC_NOERR;
    }
}

static int drv_put_varn(void *ncp, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts,
                        const void *buf, MPI_Offset bufcount, MPI_Datatype buftype, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int err = NC_NOERR, it, e2;
    void *tmp = NULL;
    const void *ptr;
    const MPI_Offset before = my_numrecs(m);
    pncx_dtype *dt = NULL;
    if (!(reqMode & NC_REQ_ZERO)) {
        err = varn_buffer(m, varid, num, counts, buf, bufcount, buftype, 1, &tmp, &ptr, &it, &dt);
        if (!err) err = pncx_nc_put_varn(m->ncid, varid, num, (const pncx_offset *const *)starts,
                                         (const pncx_offset *const *)counts, ptr, it);
        free_packed(tmp, dt);
    }
    e2 = coll_put_done(m, varid, reqMode, before);
    return (err == NC_NOERR || err == NC_ERANGE) && e2 != NC_NOERR ? e2 : err;
}

static int drv_get_varn(void *ncp, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts,
                        void *buf, MPI_Offset bufcount, MPI_Datatype buftype, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int err, it;
    void *tmp = NULL;
    const void *ptr;
    pncx_dtype *dt = NULL;
    if (reqMode & NC_REQ_ZERO) return NC_NOERR;
    err = varn_buffer(m, varid, num, counts, buf, bufcount, buftype, 0, &tmp, &ptr, &it, &dt);
    if (!err) err = pncx_nc_get_varn(m->ncid, varid, num, (const pncx_offset *const *)starts,
                                     (const pncx_offset *const *)counts, (void *)ptr, it);
    if (tmp != NULL && (err == NC_NOERR || err == NC_ERANGE)) {
        const int e2 = dt != NULL ? pncx_dev_unpack(tmp, buf, bufcount, dt, NULL)
                                  : unpack_flex(tmp, varn_nelems(m, varid, num, counts), it, buf, bufcount, buftype);
        if (e2) err = e2;
    }
    free_packed(tmp, dt);
    return err;
}

static int drv_iget_var(void *ncp, int varid, const MPI_Offset *start, const MPI_Offset *count,
                        const MPI_Offset *stride, const MPI_Offset *imap, void *buf, MPI_Offset bufcount,
                        MPI_Datatype buftype, int *reqid, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int it;
    (void)reqMode;
    if (direct_itype(m, varid, bufcount, buftype, &it) && (bufcount == -1 || buftype == MPI_DATATYPE_NULL))
        return pncx_nc_iget_varm(m->ncid, varid, start, count, stride, imap, buf, it, reqid);
    return pncx_ncmpi_iget_varm(m->ncid, varid, start, count, stride, imap, buf, bufcount, buftype, reqid);
}

static int drv_iput_var(void *ncp, int varid, const MPI_Offset *start, const MPI_Offset *count,
                        const MPI_Offset *stride, const MPI_Offset *imap, const void *buf, MPI_Offset bufcount,
                        MPI_Datatype buftype, int *reqid, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int it;
    (void)reqMode;
    if (direct_itype(m, varid, bufcount, buftype, &it) && (bufcount == -1 || buftype == MPI_DATATYPE_NULL))
        return pncx_nc_iput_varm(m->ncid, varid, start, count, stride, imap, buf, it, reqid);
    return pncx_ncmpi_iput_varm(m->ncid, varid, start, count, stride, imap, buf, bufcount, buftype, reqid);
}

static int drv_bput_var(void *ncp, int varid, const MPI_Offset *start, const MPI_Offset *count,
                        const MPI_Offset *stride, const MPI_Offset *imap, const void *buf, MPI_Offset bufcount,
                        MPI_Datatype buftype, int *reqid, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int it, err, ndims = 0, d;
    void *tmp = NULL;
    MPI_Offset want = 1;
    (void)reqMode;
    if (direct_itype(m, varid, bufcount, buftype, &it) &&
        (bufcount == -1 || buftype == MPI_DATATYPE_NULL || it != 0)) {
        if (it == 0) return NC_EBADTYPE;
        if (bufcount != -1 && buftype != MPI_DATATYPE_NULL) {
            /* a predefined buftype with an explicit bufcount must cover the
             * request exactly (ncmpio_i_getput.m4:216, dtype_decode.c:690) */
            pncx_nc_inq_var(m->ncid, varid, NULL, NULL, &ndims, NULL, NULL);
            for (d = 0; d < ndims; d++) want *= count[d];
            if (bufcount != want) return NC_EIOMISMATCH;
        }
        return pncx_nc_bput_varm(m->ncid, varid, start, count, stride, imap, buf, it, reqid);
    }
    /* derived buftype: packed now (on the device for a device buffer),
     * converted into the attached buffer now (ncmpio_i_getput.m4:266-310) */
    pncx_nc_inq_var(m->ncid, varid, NULL, NULL, &ndims, NULL, NULL);
    for (d = 0; d < ndims; d++) want *= count[d];
    if (pncx_is_device_ptr(buf)) {
        pncx_dtype *dt = NULL;
        if ((err = pack_flex_dev(buf, bufcount, buftype, want, 1, &tmp, &it, &dt)) != NC_NOERR) return err;
        err = pncx_nc_bput_varm(m->ncid, varid, start, count, stride, imap, tmp, it, reqid);
        free_packed(tmp, dt);
        return err;
    }
    if ((err = pack_flex(buf, bufcount, buftype, want, 1, &tmp, &it)) != NC_NOERR) return err;
    err = pncx_nc_bput_varm(m->ncid, varid, start, count, stride, imap, tmp, it, reqid);
    free(tmp);
    return err;
}

static int drv_iget_varn(void *ncp, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts,
                         void *buf, MPI_Offset bufcount, MPI_Datatype buftype, int *reqid, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int err, it, id = NC_REQ_NULL;
    void *tmp = NULL;
    const void *ptr;
    pncx_dtype *dt = NULL;
    (void)reqMode;
    err = varn_buffer(m, varid, num, counts, buf, bufcount, buftype, 0, &tmp, &ptr, &it, &dt);
    if (!err) err = pncx_nc_iget_varn(m->ncid, varid, num, (const pncx_offset *const *)starts,
                                      (const pncx_offset *const *)counts, (void *)ptr, it, &id);
    if (reqid) *reqid = id;
    if (tmp != NULL) {
        if (err == NC_NOERR && id != NC_REQ_NULL) err = add_stage(m, id, 1, tmp, buf, bufcount, buftype, dt);
        else free_packed(tmp, dt);
    }
    return err;
}

static int drv_iput_varn(void *ncp, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts,
                         const void *buf, MPI_Offset bufcount, MPI_Datatype buftype, int *reqid, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int err, it, id = NC_REQ_NULL;
    void *tmp = NULL;
    const void *ptr;
    pncx_dtype *dt = NULL;
    (void)reqMode;
    err = varn_buffer(m, varid, num, counts, buf, bufcount, buftype, 1, &tmp, &ptr, &it, &dt);
    if (!err) err = pncx_nc_iput_varn(m->ncid, varid, num, (const pncx_offset *const *)starts,
                                      (const pncx_offset *const *)counts, ptr, it, &id);
    if (reqid) *reqid = id;
    if (tmp != NULL) {
        if (err == NC_NOERR && id != NC_REQ_NULL) err = add_stage(m, id, 0, tmp, NULL, 0, buftype, dt);
        else free_packed(tmp, dt);
    }
    return err;
}

static int drv_bput_varn(void *ncp, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts,
                         const void *buf, MPI_Offset bufcount, MPI_Datatype buftype, int *reqid, int reqMode)
{
    NCM *m = (NCM *)ncp;
    int err, it;
    void *tmp = NULL;
    const void *ptr;
    pncx_dtype *dt = NULL;
    (void)reqMode;
    err = varn_buffer(m, varid, num, counts, buf, bufcount, buftype, 1, &tmp, &ptr, &it, &dt);
    if (!err) err = pncx_nc_bput_varn(m->ncid, varid, num, (const pncx_offset *const *)starts,
                                      (const pncx_offset *const *)counts, ptr, it, reqid);
    free_packed(tmp, dt);
    return err;
}

static int drv_buffer_attach(void *ncp, MPI_Offset bufsize)
{
    return pncx_nc_buffer_attach(((NCM *)ncp)->ncid, bufsize);
}

static int drv_buffer_detach(void *ncp)
{
    return pncx_nc_buffer_detach(((NCM *)ncp)->ncid);
}

/* ncmpio_wait (ncmpio_wait.c:808-830): the mode must match the call */
static int drv_wait(void *ncp, int num, int *reqids, int *statuses, int reqMode)
{
    NCM *m = (NCM *)ncp;
    const int coll = !(reqMode & NC_REQ_INDEP);
    int err, e2, *ids = NULL;
    MPI_Offset before;
    if (m->indef) return NC_EINDEFINE;
    if (!coll && !m->indep) return NC_ENOTINDEP;
    if (coll && m->indep) return NC_EINDEP;
    if (!coll && num == 0) return NC_NOERR;
    if (num > 0 && m->nstage > 0) {             /* the ids before wait resets them */
        ids = (int *)malloc(sizeof(int) * (size_t)num);
        if (ids == NULL) return NC_ENOMEM;
        memcpy(ids, reqids, sizeof(int) * (size_t)num);
    }
    before = my_numrecs(m);
    err = (num == 0) ? NC_NOERR : pncx_nc_wait_all(m->ncid, num, reqids, statuses);
    if (m->nstage > 0 && (num < 0 || ids != NULL)) {
        e2 = finish_stages(m, num, ids, 1);
        if (err == NC_NOERR) err = e2;
    }
    free(ids);
    if (coll) {
        /* the MAX record count over ranks, written to the file when the
         * flush created records (ncmpio_wait.c:603-672) */
        sync_numrecs_mem(m);
        if (!m->rdonly && my_numrecs(m) > before) {
            e2 = pncx_nc_sync_numrecs(m->ncid, my_numrecs(m));
            if (err == NC_NOERR) err = e2;
        }
    }
    return err;
}

static int drv_cancel(void *ncp, int num, int *reqids, int *statuses)
{
    NCM *m = (NCM *)ncp;
    int err, *ids = NULL;
    if (num > 0 && m->nstage > 0) {
        ids = (int *)malloc(sizeof(int) * (size_t)num);
        if (ids == NULL) return NC_ENOMEM;
        memcpy(ids, reqids, sizeof(int) * (size_t)num);
    }
    err = pncx_nc_cancel(m->ncid, num, reqids, statuses);
    if (m->nstage > 0 && (num < 0 || ids != NULL)) finish_stages(m, num, ids, 0);
    free(ids);
    return err;
}

/* ncmpio_driver.c:15-73, member for member */
static PNC_driver ncmi355x_driver = {
    drv_create, drv_open, drv_close, drv_enddef, drv__enddef, drv_redef, drv_sync, drv_flush, drv_abort,
    drv_set_fill, drv_inq, drv_inq_misc, drv_sync_numrecs, drv_begin_indep_data, drv_end_indep_data,
    drv_def_dim, drv_inq_dimid, drv_inq_dim, drv_rename_dim,
    drv_inq_att, drv_inq_attid, drv_inq_attname, drv_copy_att, drv_rename_att, drv_del_att, drv_get_att,
    drv_put_att,
    drv_def_var, drv_def_var_fill, drv_fill_var_rec, drv_inq_var, drv_inq_varid, drv_rename_var,
    drv_get_var, drv_put_var, drv_get_varn, drv_put_varn, drv_iget_var, drv_iput_var, drv_bput_var,
    drv_iget_varn, drv_iput_varn, drv_bput_varn, drv_buffer_attach, drv_buffer_detach, drv_wait, drv_cancel,
};

PNC_driver *ncmi355x_inq_driver(void)
{
    return &ncmi355x_driver;
}
