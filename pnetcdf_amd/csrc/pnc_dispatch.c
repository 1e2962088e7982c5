/*
 * pnc_dispatch.c -- the ncmpi_* public C API (include/pnetcdf.h) of
 * libpnetcdf.so: a restatement of PnetCDF 1.15.0's dispatcher layer
 * (src/dispatchers/file.c, dimension.c, variable.c, attribute.c,
 * attr_getput.m4, var_getput.m4) over struct PNC_driver
 * (include/pncx_dispatch.h).
 *
 * As in the reference, the dispatcher owns the ncid table and a small
 * per-file object (mode flags, the variables' shapes for argument checks),
 * validates arguments in the reference's error order (sanity_check,
 * check_start_count_stride: var_getput.m4:60-284), turns every typed entry
 * point into one driver call with a request mode (NC_REQ_WR/RD |
 * BLK/NBI/NBB | HL/FLEX | COLL/INDEP) and an MPI buftype, and leaves the
 * work to the driver -- here the MI355X driver (pnc_driver.c), which runs
 * every buffer through the HIP swap/convert kernels.
 *
 * The typed families (12 buffer types x var/var1/vara/vars/varm/varn x
 * put/get/iput/iget/bput/mput/mget x independent/collective) are
 * generated below with the preprocessor, as the reference generates them
 * with m4 (ITYPE_LIST, var_getput.m4:419-424, 810-816, 989-996).
 */
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <sys/stat.h>

#include "../../include/pncx_dispatch.h"

#define fIsSet(f, m) (((f) & (m)) != 0)

typedef struct PNC_var {
    int ndims;
    int recdim;              /* >= 0: record variable */
    nc_type xtype;
    MPI_Offset *shape;       /* [ndims] */
} PNC_var;

typedef struct PNC {
    int mode;                /* create / open mode */
    int flag;                /* NC_MODE_* */
    int format;
    char *path;
    MPI_Comm comm;
    int ndims;
    int unlimdimid;
    int nvars;
    int nrec_vars;
    PNC_var *vars;
    void *ncp;               /* driver object */
    PNC_driver *driver;
} PNC;

static PNC *pnc_list[NC_MAX_NFILES];
static int pnc_default_format = NC_FORMAT_CLASSIC;     /* file.c: ncmpi_default_create_format */
static PNC_driver *pnc_next_driver = NULL;

PNC_driver *pncx_set_driver(PNC_driver *driver)
{
    PNC_driver *old = pnc_next_driver;
    pnc_next_driver = driver;
    return old;
}

/* The ncid table is shared by every thread of the process.  The reference
 * guards it with a mutex when built with PNETCDF_THREAD_SAFE (file.c:30-33,
 * new_id_PNCList :621-648, del_from_PNCList :655-674, PNC_check_id
 * :681-703); here the mutex is always on -- the library itself runs
 * threads (warm-up, preload, I/O pool), and tests/mpi/api_check pthread
 * restates the reference's tst_pthread.c on it. */
static pthread_mutex_t pnc_lock = PTHREAD_MUTEX_INITIALIZER;

/* PNC_check_id (file.c) */
static int PNC_check_id(int ncid, PNC **pncp)
{
    int err = NC_NOERR;
    if (ncid < 0 || ncid >= NC_MAX_NFILES) return NC_EBADID;
    pthread_mutex_lock(&pnc_lock);
    if (pnc_list[ncid] == NULL) err = NC_EBADID;
    else *pncp = pnc_list[ncid];
    pthread_mutex_unlock(&pnc_lock);
    return err;
}

static int new_id(PNC *p, int *ncidp)
{
    int i, err = NC_ENFILE;
    pthread_mutex_lock(&pnc_lock);
    for (i = 0; i < NC_MAX_NFILES; i++)
        if (pnc_list[i] == NULL) {
            pnc_list[i] = p;
            *ncidp = i;
            err = NC_NOERR;
            break;
        }
    pthread_mutex_unlock(&pnc_lock);
    return err;
}

static void del_id(int ncid)
{
    pthread_mutex_lock(&pnc_lock);
    pnc_list[ncid] = NULL;
    pthread_mutex_unlock(&pnc_lock);
}

static void free_pnc(PNC *p)
{
    int i;
    if (p == NULL) return;
    for (i = 0; i < p->nvars; i++) free(p->vars[i].shape);
    free(p->vars);
    free(p->path);
    if (p->comm != MPI_COMM_NULL) MPI_Comm_free(&p->comm);
    free(p);
}

/* NC_MODE_SAFE / NC_MODE_STRICT_COORD_BOUND from the environment (file.c:843-878) */
static void set_env_mode(int *env_mode)
{
    const char *s = getenv("PNETCDF_SAFE_MODE");
    if (s != NULL && *s == '1') *env_mode |= NC_MODE_SAFE;
    s = getenv("PNETCDF_RELAX_COORD_BOUND");
    if (s != NULL && *s == '0') *env_mode |= NC_MODE_STRICT_COORD_BOUND;
#if PNETCDF_RELAX_COORD_BOUND == 0
    if (s == NULL) *env_mode |= NC_MODE_STRICT_COORD_BOUND;
#endif
}

/* the dispatcher's copy of one variable's shape (file.c:1550-1590) */
static int add_var(PNC *p, int varid)
{
    int ndims = 0, j, err, *dimids;
    nc_type xtype;
    PNC_var *v;
    if (varid != p->nvars) return NC_EINTERNAL;
    if ((err = p->driver->inq_var(p->ncp, varid, NULL, &xtype, &ndims, NULL, NULL, NULL, NULL, NULL)))
        return err;
    v = (PNC_var *)realloc(p->vars, sizeof(PNC_var) * (size_t)(p->nvars + 1));
    if (v == NULL) return NC_ENOMEM;
    p->vars = v;
    v = &p->vars[p->nvars];
    v->ndims = ndims;
    v->xtype = xtype;
    v->recdim = -1;
    v->shape = NULL;
    if (ndims > 0) {
        dimids = (int *)malloc(sizeof(int) * (size_t)ndims);
        v->shape = (MPI_Offset *)malloc(sizeof(MPI_Offset) * (size_t)ndims);
        if (dimids == NULL || v->shape == NULL) { free(dimids); free(v->shape); return NC_ENOMEM; }
        err = p->driver->inq_var(p->ncp, varid, NULL, NULL, NULL, dimids, NULL, NULL, NULL, NULL);
        for (j = 0; j < ndims && !err; j++) {
            err = p->driver->inq_dim(p->ncp, dimids[j], NULL, &v->shape[j]);
            if (dimids[j] == p->unlimdimid) v->recdim = j;
        }
        free(dimids);
        if (err) { free(v->shape); return err; }
    }
    if (v->recdim >= 0) p->nrec_vars++;
    p->nvars++;
    return NC_NOERR;
}

/* ------------------------------------------------------------------------ */
/* error strings (error_codes.c): this library's own wording               */
/* ------------------------------------------------------------------------ */
const char *ncmpi_strerror(int err)
{
    static char unknown[64];
    if (err > 0) return strerror(err);                         /* system errno */
    switch (err) {
    case NC_NOERR: return "No error";
    case NC_EBADID: return "NetCDF: Not a valid ID";
    case NC_ENFILE: return "NetCDF: Too many files open";
    case NC_EEXIST: return "NetCDF: File exists && NC_NOCLOBBER";
    case NC_EINVAL: return "NetCDF: Invalid argument";
    case NC_EPERM: return "NetCDF: Write to read only";
    case NC_ENOTINDEFINE: return "NetCDF: Operation not allowed in data mode";
    case NC_EINDEFINE: return "NetCDF: Operation not allowed in define mode";
    case NC_EINVALCOORDS: return "NetCDF: Index exceeds dimension bound";
    case NC_EMAXDIMS: return "NetCDF: NC_MAX_DIMS exceeded";
    case NC_ENAMEINUSE: return "NetCDF: String match to name in use";
    case NC_ENOTATT: return "NetCDF: Attribute not found";
    case NC_EMAXATTS: return "NetCDF: NC_MAX_ATTRS exceeded";
    case NC_EBADTYPE: return "NetCDF: Not a valid data type or _FillValue type mismatch";
    case NC_EBADDIM: return "NetCDF: Invalid dimension ID or name";
    case NC_EUNLIMPOS: return "NetCDF: NC_UNLIMITED in the wrong index";
    case NC_EMAXVARS: return "NetCDF: NC_MAX_VARS exceeded";
    case NC_ENOTVAR: return "NetCDF: Variable not found";
    case NC_EGLOBAL: return "NetCDF: Action prohibited on NC_GLOBAL varid";
    case NC_ENOTNC: return "NetCDF: Unknown file format";
    case NC_ESTS: return "NetCDF: In Fortran, string too short";
    case NC_EMAXNAME: return "NetCDF: NC_MAX_NAME exceeded";
    case NC_EUNLIMIT: return "NetCDF: NC_UNLIMITED size already in use";
    case NC_ENORECVARS: return "NetCDF: nc_rec op when there are no record vars";
    case NC_ECHAR: return "NetCDF: Attempt to convert between text & numbers";
    case NC_EEDGE: return "NetCDF: Start+count exceeds dimension bound";
    case NC_ESTRIDE: return "NetCDF: Illegal stride";
    case NC_EBADNAME: return "NetCDF: Name contains illegal characters";
    case NC_ERANGE: return "NetCDF: Numeric conversion not representable";
    case NC_ENOMEM: return "NetCDF: Memory allocation (malloc) failure";
    case NC_EVARSIZE: return "NetCDF: One or more variable sizes violate format constraints";
    case NC_EDIMSIZE: return "NetCDF: Invalid dimension size";
    case NC_ETRUNC: return "NetCDF: File likely truncated or possibly corrupted";
    case NC_EAXISTYPE: return "NetCDF: Illegal axis type";
    case NC_EIO: return "NetCDF: I/O failure";
    case NC_ENOTFOUND: return "NetCDF: No such file";
    case NC_EINTERNAL: return "NetCDF: Internal library error";
    case NC_ENOTNC3: return "NetCDF: Attempting netcdf-3 operation on netcdf-4 file";
    case NC_ENOTBUILT: return "NetCDF: Attempt to use feature that was not turned on when the library was built";
    case NC_EMPI: return "NetCDF: MPI operation failed";
    case NC_ENULLPAD: return "NetCDF: File header is not null-byte padded";
    case NC_ESMALL: return "Size of MPI_Offset or MPI_Aint too small for requested format";
    case NC_ENOTINDEP: return "Operation not allowed in collective data mode";
    case NC_EINDEP: return "Operation not allowed in independent data mode";
    case NC_EFILE: return "Unknown error in file operation";
    case NC_EREAD: return "Unknown error in reading file";
    case NC_EWRITE: return "Unknown error in writing to file";
    case NC_EOFILE: return "Can not open/create file";
    case NC_EMULTITYPES: return "Multiple element types used in an MPI derived data type";
    case NC_EIOMISMATCH: return "Input/Output data amount mismatch";
    case NC_ENEGATIVECNT: return "Negative count is prohibited";
    case NC_EUNSPTETYPE: return "Unsupported element type in an MPI derived data type";
    case NC_EINVAL_REQUEST: return "Invalid nonblocking request ID";
    case NC_EAINT_TOO_SMALL: return "MPI_Aint not large enough to hold the requested value";
    case NC_ENOTSUPPORT: return "Feature is not yet supported";
    case NC_ENULLBUF: return "Trying to attach a NULL buffer";
    case NC_EPREVATTACHBUF: return "A buffer is already attached";
    case NC_ENULLABUF: return "No attached buffer";
    case NC_EPENDINGBPUT: return "Pending bput requests: the buffer cannot be detached";
    case NC_EINSUFFBUF: return "Attached buffer is too small";
    case NC_ENOENT: return "File does not exist";
    case NC_EINTOVERFLOW: return "Overflow when casting to a 4-byte integer";
    case NC_ENOTENABLED: return "Feature is not enabled";
    case NC_EBAD_FILE: return "Invalid file name";
    case NC_ENO_SPACE: return "Not enough space";
    case NC_EQUOTA: return "Disk quota exceeded";
    case NC_ENULLSTART: return "Argument start is a NULL pointer";
    case NC_ENULLCOUNT: return "Argument count is a NULL pointer";
    case NC_EINVAL_CMODE: return "Invalid file create mode";
    case NC_ETYPESIZE: return "MPI derived data type size error";
    case NC_ETYPE_MISMATCH: return "Element type of the MPI derived data type mismatches the variable type";
    case NC_ETYPESIZE_MISMATCH: return "File type size mismatches buffer type size";
    case NC_ESTRICTCDF2: return "Attempting a CDF-5 operation on a CDF-1 or CDF-2 file";
    case NC_ENOTRECVAR: return "Attempting an operation meant for record variables only";
    case NC_ENOTFILL: return "Attempting to fill a variable whose fill mode is off";
    case NC_EINVAL_OMODE: return "Invalid file open mode";
    case NC_EPENDING: return "Pending nonblocking requests at file close";
    case NC_EMAX_REQ: return "Size of an I/O request exceeds INT_MAX";
    case NC_EBADLOG: return "Unrecognized burst-buffer log file format";
    case NC_EFLUSHED: return "Nonblocking request already flushed: too late to cancel";
    case NC_EADIOS: return "Unknown ADIOS error";
    case NC_EFSTYPE: return "File system type not supported";
    case NC_EDRIVER: return "Invalid PnetCDF I/O driver";
    case NC_EFILEVIEW: return "File view is not monotonically non-decreasing";
    case NC_EMULTIDEFINE: return "File header is inconsistent among processes";
    case NC_EMULTIDEFINE_OMODE: return "File open modes are inconsistent among processes";
    case NC_EMULTIDEFINE_DIM_NUM: return "Number of dimensions is defined inconsistently among processes";
    case NC_EMULTIDEFINE_DIM_SIZE: return "Dimension size is defined inconsistently among processes";
    case NC_EMULTIDEFINE_DIM_NAME: return "Dimension name is defined inconsistently among processes";
    case NC_EMULTIDEFINE_VAR_NUM: return "Number of variables is defined inconsistently among processes";
    case NC_EMULTIDEFINE_VAR_NAME: return "Variable name is defined inconsistently among processes";
    case NC_EMULTIDEFINE_VAR_NDIMS: return "Dimensionality of a variable is defined inconsistently";
    case NC_EMULTIDEFINE_VAR_DIMIDS: return "Dimension IDs of a variable are defined inconsistently";
    case NC_EMULTIDEFINE_VAR_TYPE: return "Data type of a variable is defined inconsistently";
    case NC_EMULTIDEFINE_VAR_LEN: return "Number of elements of a variable is defined inconsistently";
    case NC_EMULTIDEFINE_NUMRECS: return "Number of records is inconsistent among processes";
    case NC_EMULTIDEFINE_VAR_BEGIN: return "Variable file offset is inconsistent among processes";
    case NC_EMULTIDEFINE_ATTR_NUM: return "Number of attributes is defined inconsistently";
    case NC_EMULTIDEFINE_ATTR_SIZE: return "Attribute size is inconsistent among processes";
    case NC_EMULTIDEFINE_ATTR_NAME: return "Attribute name is defined inconsistently";
    case NC_EMULTIDEFINE_ATTR_TYPE: return "Attribute type is defined inconsistently";
    case NC_EMULTIDEFINE_ATTR_LEN: return "Attribute length is defined inconsistently";
    case NC_EMULTIDEFINE_ATTR_VAL: return "Attribute value is defined inconsistently";
    case NC_EMULTIDEFINE_FNC_ARGS: return "Arguments of a collective call are inconsistent among processes";
    case NC_EMULTIDEFINE_FILL_MODE: return "File fill mode is inconsistent among processes";
    case NC_EMULTIDEFINE_VAR_FILL_MODE: return "Variable fill mode is inconsistent among processes";
    case NC_EMULTIDEFINE_VAR_FILL_VALUE: return "Variable fill value is inconsistent among processes";
    case NC_EMULTIDEFINE_CMODE: return "File create modes are inconsistent among processes";
    case NC_EMULTIDEFINE_HINTS: return "I/O hints are inconsistent among processes";
    case -1900: return "MI355X: GPU runtime failure or no GPU visible (the conversion has no CPU path)";
    default:
        snprintf(unknown, sizeof unknown, "Unknown error code %d", err);
        return unknown;
    }
}

/* the error code's name (error_codes.c ncmpi_strerrno) */
const char *ncmpi_strerrno(int err)
{
    static char unknown[32];
#define E(c) case c: return #c;
    switch (err) {
    E(NC_NOERR) E(NC_EBADID) E(NC_ENFILE) E(NC_EEXIST) E(NC_EINVAL) E(NC_EPERM) E(NC_ENOTINDEFINE)
    E(NC_EINDEFINE) E(NC_EINVALCOORDS) E(NC_EMAXDIMS) E(NC_ENAMEINUSE) E(NC_ENOTATT) E(NC_EMAXATTS)
    E(NC_EBADTYPE) E(NC_EBADDIM) E(NC_EUNLIMPOS) E(NC_EMAXVARS) E(NC_ENOTVAR) E(NC_EGLOBAL) E(NC_ENOTNC)
    E(NC_ESTS) E(NC_EMAXNAME) E(NC_EUNLIMIT) E(NC_ENORECVARS) E(NC_ECHAR) E(NC_EEDGE) E(NC_ESTRIDE)
    E(NC_EBADNAME) E(NC_ERANGE) E(NC_ENOMEM) E(NC_EVARSIZE) E(NC_EDIMSIZE) E(NC_ETRUNC) E(NC_EAXISTYPE)
    E(NC_EIO) E(NC_ENOTFOUND) E(NC_EINTERNAL) E(NC_ENOTNC3) E(NC_ENOTBUILT) E(NC_EMPI) E(NC_ENULLPAD)
    E(NC_ESMALL) E(NC_ENOTINDEP) E(NC_EINDEP) E(NC_EFILE) E(NC_EREAD) E(NC_EWRITE) E(NC_EOFILE)
    E(NC_EMULTITYPES) E(NC_EIOMISMATCH) E(NC_ENEGATIVECNT) E(NC_EUNSPTETYPE) E(NC_EINVAL_REQUEST)
    E(NC_EAINT_TOO_SMALL) E(NC_ENOTSUPPORT) E(NC_ENULLBUF) E(NC_EPREVATTACHBUF) E(NC_ENULLABUF)
    E(NC_EPENDINGBPUT) E(NC_EINSUFFBUF) E(NC_ENOENT) E(NC_EINTOVERFLOW) E(NC_ENOTENABLED) E(NC_EBAD_FILE)
    E(NC_ENO_SPACE) E(NC_EQUOTA) E(NC_ENULLSTART) E(NC_ENULLCOUNT) E(NC_EINVAL_CMODE) E(NC_ETYPESIZE)
    E(NC_ETYPE_MISMATCH) E(NC_ETYPESIZE_MISMATCH) E(NC_ESTRICTCDF2) E(NC_ENOTRECVAR) E(NC_ENOTFILL)
    E(NC_EINVAL_OMODE) E(NC_EPENDING) E(NC_EMAX_REQ) E(NC_EBADLOG) E(NC_EFLUSHED) E(NC_EADIOS)
    E(NC_EFSTYPE) E(NC_EDRIVER) E(NC_EFILEVIEW) E(NC_EMULTIDEFINE) E(NC_EMULTIDEFINE_OMODE)
    E(NC_EMULTIDEFINE_CMODE)
    default:
        snprintf(unknown, sizeof unknown, "Unknown code %d", err);
        return unknown;
    }
#undef E
}

const char *ncmpi_inq_libvers(void)
{
    return "version = " PNETCDF_VERSION " of MI355X (HIP conversion path, gfx950)";
}

/* ------------------------------------------------------------------------ */
/* files (file.c)                                                            */
/* ------------------------------------------------------------------------ */
static PNC *new_pnc(MPI_Comm comm, const char *path, int *err)
{
    PNC *p = (PNC *)calloc(1, sizeof *p);
    *err = NC_NOERR;
    if (p == NULL) { *err = NC_ENOMEM; return NULL; }
    p->comm = MPI_COMM_NULL;
    p->unlimdimid = -1;
    /* the dispatcher's own communicator (file.c:919-933) */
    if (MPI_Comm_dup(comm, &p->comm) != MPI_SUCCESS) { *err = NC_EMPI; free(p); return NULL; }
    if (path == NULL || *path == '\0') { *err = NC_EBAD_FILE; return p; }
    p->path = strdup(path);
    if (p->path == NULL) *err = NC_ENOMEM;
    return p;
}

static PNC_comm_attr no_ina(void)
{
    PNC_comm_attr a;
    memset(&a, 0, sizeof a);
    a.numa_comm = a.ina_inter_comm = a.ina_intra_comm = MPI_COMM_NULL;
    return a;
}

int ncmpi_create(MPI_Comm comm, const char *path, int cmode, MPI_Info info, int *ncidp)
{
    int err, status = NC_NOERR, env_mode = 0, rank, nprocs, format;
    void *ncp = NULL;
    PNC *p;
    PNC_driver *driver;
    if (ncidp == NULL) return NC_EINVAL;
    *ncidp = -1;
    p = new_pnc(comm, path, &err);
    if (err) { free_pnc(p); return err; }
    MPI_Comm_rank(p->comm, &rank);
    MPI_Comm_size(p->comm, &nprocs);
    if (rank == 0) set_env_mode(&env_mode);
    if (nprocs > 1) {               /* root's cmode is used; report a mismatch (file.c:960-983) */
        int modes[2] = {cmode, env_mode};
        MPI_Bcast(modes, 2, MPI_INT, 0, p->comm);
        if (modes[0] != cmode) { cmode = modes[0]; status = NC_EMULTIDEFINE_CMODE; }
        env_mode = modes[1];
    }
    if (cmode & NC_NETCDF4) { free_pnc(p); return NC_ENOTBUILT; }            /* file.c:1073-1078 */
    if ((cmode & (NC_64BIT_OFFSET | NC_64BIT_DATA)) == (NC_64BIT_OFFSET | NC_64BIT_DATA)) {
        free_pnc(p);
        return NC_EINVAL_CMODE;
    }
    if (cmode & NC_64BIT_DATA) format = NC_FORMAT_CDF5;
    else if (cmode & NC_64BIT_OFFSET) format = NC_FORMAT_CDF2;
    else if (cmode & NC_CLASSIC_MODEL) format = NC_FORMAT_CLASSIC;
    else {                           /* the default format (file.c:1098-1111) */
        format = pnc_default_format;
        if (format == NC_FORMAT_CDF5) cmode |= NC_64BIT_DATA;
        else if (format == NC_FORMAT_CDF2) cmode |= NC_64BIT_OFFSET;
        else if (format == NC_FORMAT_NETCDF4 || format == NC_FORMAT_NETCDF4_CLASSIC) {
            free_pnc(p);
            return NC_ENOTBUILT;
        }
    }
    driver = pnc_next_driver ? pnc_next_driver : ncmi355x_inq_driver();
    p->flag = NC_MODE_DEF | NC_MODE_CREATE | env_mode;
    if ((err = new_id(p, ncidp)) != NC_NOERR) { free_pnc(p); return err; }
    err = driver->create(p->comm, p->path, cmode, *ncidp, env_mode, info, no_ina(), &ncp);
    if (status == NC_NOERR) status = err;
    if (err != NC_NOERR) {
        del_id(*ncidp);
        *ncidp = -1;
        free_pnc(p);
        return status;
    }
    p->mode = cmode;
    p->driver = driver;
    p->ncp = ncp;
    p->format = format;
    return status;
}

int ncmpi_open(MPI_Comm comm, const char *path, int omode, MPI_Info info, int *ncidp)
{
    int err, status = NC_NOERR, env_mode = 0, rank, nprocs, format, i, nvars = 0;
    void *ncp = NULL;
    PNC *p;
    PNC_driver *driver;
    if (ncidp == NULL) return NC_EINVAL;
    *ncidp = -1;
    p = new_pnc(comm, path, &err);
    if (err) { free_pnc(p); return err; }
    MPI_Comm_rank(p->comm, &rank);
    MPI_Comm_size(p->comm, &nprocs);
    if (rank == 0) set_env_mode(&env_mode);
    if (nprocs > 1) {
        int modes[2] = {omode, env_mode};
        MPI_Bcast(modes, 2, MPI_INT, 0, p->comm);
        if (modes[0] != omode) { omode = modes[0]; status = NC_EMULTIDEFINE_OMODE; }
        env_mode = modes[1];
    }
    /* the format decides the driver (file.c:1420-1470): classic only here */
    err = NC_NOERR;
    if (rank == 0) err = ncmpi_inq_file_format(path, &format);
    if (nprocs > 1) {
        int v[2] = {err, format};
        MPI_Bcast(v, 2, MPI_INT, 0, p->comm);
        err = v[0];
        format = v[1];
    }
    if (err == NC_NOERR && format == NC_FORMAT_UNKNOWN) err = NC_ENOTNC;
    if (err == NC_NOERR && (format == NC_FORMAT_NETCDF4 || format == NC_FORMAT_NETCDF4_CLASSIC)) err = NC_ENOTBUILT;
    if (err) { free_pnc(p); return err; }
    driver = pnc_next_driver ? pnc_next_driver : ncmi355x_inq_driver();
    p->flag = env_mode;
    if (!(omode & NC_WRITE)) p->flag |= NC_MODE_RDONLY;
    if ((err = new_id(p, ncidp)) != NC_NOERR) { free_pnc(p); return err; }
    err = driver->open(p->comm, p->path, omode, *ncidp, env_mode, info, no_ina(), &ncp);
    if (status == NC_NOERR) status = err;
    if (err != NC_NOERR) {
        del_id(*ncidp);
        *ncidp = -1;
        free_pnc(p);
        return status;
    }
    p->mode = omode;
    p->driver = driver;
    p->ncp = ncp;
    p->format = format;
    /* the variables' shapes for argument checks (file.c:1540-1595) */
    err = driver->inq(ncp, &p->ndims, &nvars, NULL, &p->unlimdimid);
    for (i = 0; i < nvars && !err; i++) err = add_var(p, i);
    if (err) {
        driver->close(ncp);
        del_id(*ncidp);
        *ncidp = -1;
        free_pnc(p);
        return err;
    }
    return status;
}

int ncmpi_close(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    err = p->driver->close(p->ncp);
    del_id(ncid);                   /* removed even on error (file.c:1716) */
    free_pnc(p);
    return err;
}

int ncmpi_abort(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    err = p->driver->abort(p->ncp);
    del_id(ncid);
    free_pnc(p);
    return err;
}

int ncmpi_delete(const char *filename, MPI_Info info)
{
    (void)info;
    if (filename == NULL || *filename == '\0') return NC_EBAD_FILE;
    if (unlink(filename) != 0) return errno == ENOENT ? NC_ENOENT : NC_EFILE;
    return NC_NOERR;
}

static int enddef_common(PNC *p, int err)
{
    if (p->flag & NC_MODE_SAFE) {
        int minE;
        MPI_Allreduce(&err, &minE, 1, MPI_INT, MPI_MIN, p->comm);
        return minE;
    }
    return err;
}

int ncmpi_enddef(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (!(p->flag & NC_MODE_DEF)) err = NC_ENOTINDEFINE;
    if ((err = enddef_common(p, err)) != NC_NOERR) return err;
    if ((err = p->driver->enddef(p->ncp)) != NC_NOERR) return err;
    p->flag &= ~(NC_MODE_INDEP | NC_MODE_DEF | NC_MODE_CREATE);   /* collective data mode */
    return NC_NOERR;
}

int ncmpi__enddef(int ncid, MPI_Offset h_minfree, MPI_Offset v_align, MPI_Offset v_minfree, MPI_Offset r_align)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (!(p->flag & NC_MODE_DEF)) err = NC_ENOTINDEFINE;
    if (!err && (h_minfree < 0 || v_align < 0 || v_minfree < 0 || r_align < 0)) err = NC_EINVAL;
    if ((err = enddef_common(p, err)) != NC_NOERR) return err;
    if ((err = p->driver->_enddef(p->ncp, h_minfree, v_align, v_minfree, r_align)) != NC_NOERR) return err;
    p->flag &= ~(NC_MODE_INDEP | NC_MODE_DEF | NC_MODE_CREATE);
    return NC_NOERR;
}

int ncmpi_redef(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;                 /* file.c:1851-1858 */
    if (p->flag & NC_MODE_DEF) return NC_EINDEFINE;
    if ((err = p->driver->redef(p->ncp)) != NC_NOERR) return err;
    p->flag |= NC_MODE_DEF;
    return NC_NOERR;
}

int ncmpi_sync(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->sync(p->ncp);
}

int ncmpi_flush(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->flush(p->ncp);
}

int ncmpi_sync_numrecs(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->sync_numrecs(p->ncp);
}

int ncmpi_begin_indep_data(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if ((err = p->driver->begin_indep_data(p->ncp)) != NC_NOERR) return err;
    p->flag |= NC_MODE_INDEP;
    return NC_NOERR;
}

int ncmpi_end_indep_data(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if ((err = p->driver->end_indep_data(p->ncp)) != NC_NOERR) return err;
    p->flag &= ~NC_MODE_INDEP;
    return NC_NOERR;
}

int ncmpi_set_fill(int ncid, int fillmode, int *old_modep)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;                 /* file.c:1951-1957 */
    if (!(p->flag & NC_MODE_DEF)) return NC_ENOTINDEFINE;
    if ((err = p->driver->set_fill(p->ncp, fillmode, old_modep)) != NC_NOERR) return err;
    if (fillmode == NC_FILL) p->flag |= NC_MODE_FILL;
    else p->flag &= ~NC_MODE_FILL;
    return NC_NOERR;
}

int ncmpi_set_default_format(int format, int *old_formatp)
{
    if (old_formatp != NULL) *old_formatp = pnc_default_format;
    if (format != NC_FORMAT_CLASSIC && format != NC_FORMAT_CDF2 && format != NC_FORMAT_NETCDF4 &&
        format != NC_FORMAT_NETCDF4_CLASSIC && format != NC_FORMAT_CDF5)
        return NC_EINVAL;
    pnc_default_format = format;
    return NC_NOERR;
}

int ncmpi_inq_default_format(int *formatp)
{
    if (formatp == NULL) return NC_EINVAL;
    *formatp = pnc_default_format;
    return NC_NOERR;
}

/* the file's format from its magic bytes (file.c:2026-2160) */
int ncmpi_inq_file_format(const char *filename, int *formatp)
{
    static const unsigned char hdf5[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
    unsigned char sig[8];
    FILE *fp;
    long off = 0;
    size_t r;
    if (filename == NULL || *filename == '\0') return NC_EBAD_FILE;
    if (formatp == NULL) return NC_NOERR;
    *formatp = NC_FORMAT_UNKNOWN;
    fp = fopen(filename, "rb");
    if (fp == NULL) return errno == ENOENT ? NC_ENOENT : errno == ENAMETOOLONG ? NC_EBAD_FILE : NC_EFILE;
    r = fread(sig, 1, 8, fp);
    if (r < 4) { fclose(fp); return NC_NOERR; }
    if (memcmp(sig, "CDF", 3) == 0) {
        if (sig[3] == 1) *formatp = NC_FORMAT_CLASSIC;
        else if (sig[3] == 2) *formatp = NC_FORMAT_CDF2;
        else if (sig[3] == 5) *formatp = NC_FORMAT_CDF5;
    } else {
        while (r == 8 && memcmp(sig, hdf5, 8) != 0) {       /* HDF5 superblock at 0, 512, 1024, ... */
            off = off == 0 ? 512 : off * 2;
            if (fseek(fp, off, SEEK_SET) != 0) break;
            r = fread(sig, 1, 8, fp);
        }
        if (r == 8 && memcmp(sig, hdf5, 8) == 0) *formatp = NC_FORMAT_NETCDF4;
    }
    fclose(fp);
    return NC_NOERR;
}

int ncmpi_inq_format(int ncid, int *formatp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (formatp) *formatp = p->format;
    return NC_NOERR;
}

int ncmpi_inq_version(int ncid, int *nc_mode)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (nc_mode == NULL) return NC_NOERR;
    if (p->format == NC_FORMAT_CDF5) *nc_mode = NC_64BIT_DATA;
    else if (p->format == NC_FORMAT_CDF2) *nc_mode = NC_64BIT_OFFSET;
    else *nc_mode = NC_CLASSIC_MODEL;
    return NC_NOERR;
}

int ncmpi_inq(int ncid, int *ndimsp, int *nvarsp, int *ngattsp, int *unlimdimidp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->inq(p->ncp, ndimsp, nvarsp, ngattsp, unlimdimidp);
}

int ncmpi_inq_ndims(int ncid, int *ndimsp) { return ncmpi_inq(ncid, ndimsp, NULL, NULL, NULL); }
int ncmpi_inq_nvars(int ncid, int *nvarsp) { return ncmpi_inq(ncid, NULL, nvarsp, NULL, NULL); }
int ncmpi_inq_natts(int ncid, int *ngattsp) { return ncmpi_inq(ncid, NULL, NULL, ngattsp, NULL); }
int ncmpi_inq_unlimdim(int ncid, int *unlimdimidp) { return ncmpi_inq(ncid, NULL, NULL, NULL, unlimdimidp); }

#define INQ_MISC(ncid, ...)                                                               \
    PNC *p;                                                                              \
    int err = PNC_check_id(ncid, &p);                                                    \
    if (err) return err;                                                                 \
    return p->driver->inq_misc(p->ncp, __VA_ARGS__)

int ncmpi_inq_path(int ncid, int *pathlen, char *path)
{ INQ_MISC(ncid, pathlen, path, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_num_fix_vars(int ncid, int *n)
{ INQ_MISC(ncid, NULL, NULL, n, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_num_rec_vars(int ncid, int *n)
{ INQ_MISC(ncid, NULL, NULL, NULL, n, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_striping(int ncid, int *striping_size, int *striping_count)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, striping_size, striping_count, NULL, NULL, NULL, NULL, NULL, NULL, NULL,
           NULL, NULL); }
int ncmpi_inq_header_size(int ncid, MPI_Offset *size)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, size, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_header_extent(int ncid, MPI_Offset *extent)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, extent, NULL, NULL, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_recsize(int ncid, MPI_Offset *recsize)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, recsize, NULL, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_put_size(int ncid, MPI_Offset *size)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, size, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_get_size(int ncid, MPI_Offset *size)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, size, NULL, NULL, NULL, NULL); }
int ncmpi_inq_file_info(int ncid, MPI_Info *info_used)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, info_used, NULL, NULL, NULL); }
int ncmpi_get_file_info(int ncid, MPI_Info *info_used) { return ncmpi_inq_file_info(ncid, info_used); }
int ncmpi_inq_nreqs(int ncid, int *nreqs)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, nreqs, NULL, NULL); }
int ncmpi_inq_buffer_usage(int ncid, MPI_Offset *usage)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, usage, NULL); }
int ncmpi_inq_buffer_size(int ncid, MPI_Offset *buf_size)
{ INQ_MISC(ncid, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, buf_size); }

/* malloc tracing is a build option of the reference (PNC_MALLOC_TRACE), off here */
int ncmpi_inq_malloc_size(MPI_Offset *size) { (void)size; return NC_ENOTENABLED; }
int ncmpi_inq_malloc_max_size(MPI_Offset *size) { (void)size; return NC_ENOTENABLED; }
int ncmpi_inq_malloc_list(void) { return NC_ENOTENABLED; }

int ncmpi_inq_files_opened(int *num, int *ncids)
{
    int i;
    if (num == NULL) return NC_EINVAL;
    *num = 0;
    pthread_mutex_lock(&pnc_lock);
    for (i = 0; i < NC_MAX_NFILES; i++)
        if (pnc_list[i] != NULL) {
            if (ncids != NULL) ncids[*num] = i;
            (*num)++;
        }
    pthread_mutex_unlock(&pnc_lock);
    return NC_NOERR;
}

int ncmpi_buffer_attach(int ncid, MPI_Offset bufsize)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->buffer_attach(p->ncp, bufsize);
}

int ncmpi_buffer_detach(int ncid)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->buffer_detach(p->ncp);
}

int ncmpi_wait(int ncid, int count, int array_of_requests[], int array_of_statuses[])
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->wait(p->ncp, count, array_of_requests, array_of_statuses, NC_REQ_INDEP);
}

int ncmpi_wait_all(int ncid, int count, int array_of_requests[], int array_of_statuses[])
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->wait(p->ncp, count, array_of_requests, array_of_statuses, NC_REQ_COLL);
}

int ncmpi_cancel(int ncid, int num, int *reqs, int *statuses)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    return p->driver->cancel(p->ncp, num, reqs, statuses);
}

/* ------------------------------------------------------------------------ */
/* dimensions (dimension.c)                                                  */
/* ------------------------------------------------------------------------ */
int ncmpi_def_dim(int ncid, const char *name, MPI_Offset len, int *idp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p), dimid = -1;
    if (err) return err;
    if (!(p->flag & NC_MODE_DEF)) return NC_ENOTINDEFINE;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    if (len < 0) return NC_EDIMSIZE;
    if ((err = p->driver->def_dim(p->ncp, name, len, &dimid)) != NC_NOERR) return err;
    if (len == NC_UNLIMITED) p->unlimdimid = dimid;
    p->ndims++;
    if (idp) *idp = dimid;
    return NC_NOERR;
}

int ncmpi_inq_dimid(int ncid, const char *name, int *idp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    return p->driver->inq_dimid(p->ncp, name, idp);
}

int ncmpi_inq_dim(int ncid, int dimid, char *name, MPI_Offset *lenp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (dimid < 0 || dimid >= p->ndims) return NC_EBADDIM;
    return p->driver->inq_dim(p->ncp, dimid, name, lenp);
}

int ncmpi_inq_dimname(int ncid, int dimid, char *name) { return ncmpi_inq_dim(ncid, dimid, name, NULL); }
int ncmpi_inq_dimlen(int ncid, int dimid, MPI_Offset *lenp) { return ncmpi_inq_dim(ncid, dimid, NULL, lenp); }

int ncmpi_rename_dim(int ncid, int dimid, const char *name)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;
    if (dimid < 0 || dimid >= p->ndims) return NC_EBADDIM;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    return p->driver->rename_dim(p->ncp, dimid, name);
}

/* ------------------------------------------------------------------------ */
/* variables (variable.c)                                                    */
/* ------------------------------------------------------------------------ */
int ncmpi_def_var(int ncid, const char *name, nc_type xtype, int ndims, const int *dimidsp, int *varidp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p), varid = -1;
    if (err) return err;
    if (!(p->flag & NC_MODE_DEF)) return NC_ENOTINDEFINE;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    if (xtype < NC_BYTE || xtype > NC_UINT64) return NC_EBADTYPE;
    if (p->format != NC_FORMAT_CDF5 && xtype > NC_DOUBLE) return NC_ESTRICTCDF2;
    if (ndims < 0) return NC_EINVAL;
    if (ndims > 0 && dimidsp == NULL) return NC_EINVAL;
    if ((err = p->driver->def_var(p->ncp, name, xtype, ndims, dimidsp, &varid)) != NC_NOERR) return err;
    if ((err = add_var(p, varid)) != NC_NOERR) return err;
    if (varidp) *varidp = varid;
    return NC_NOERR;
}

int ncmpi_def_var_fill(int ncid, int varid, int no_fill, const void *fill_value)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;
    if (!(p->flag & NC_MODE_DEF)) return NC_ENOTINDEFINE;
    if (varid == NC_GLOBAL) return NC_EGLOBAL;
    if (varid < 0 || varid >= p->nvars) return NC_ENOTVAR;
    return p->driver->def_var_fill(p->ncp, varid, no_fill, fill_value);
}

int ncmpi_inq_var_fill(int ncid, int varid, int *no_fill, void *fill_value)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (varid == NC_GLOBAL) return NC_EGLOBAL;
    if (varid < 0 || varid >= p->nvars) return NC_ENOTVAR;
    return p->driver->inq_var(p->ncp, varid, NULL, NULL, NULL, NULL, NULL, NULL, no_fill, fill_value);
}

int ncmpi_fill_var_rec(int ncid, int varid, MPI_Offset recno)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;
    if (p->flag & NC_MODE_DEF) return NC_EINDEFINE;
    if (varid == NC_GLOBAL) return NC_EGLOBAL;
    if (varid < 0 || varid >= p->nvars) return NC_ENOTVAR;
    if (p->vars[varid].recdim < 0) return NC_ENOTRECVAR;
    return p->driver->fill_var_rec(p->ncp, varid, recno);
}

int ncmpi_rename_var(int ncid, int varid, const char *name)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;
    if (varid == NC_GLOBAL) return NC_EGLOBAL;
    if (varid < 0 || varid >= p->nvars) return NC_ENOTVAR;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    return p->driver->rename_var(p->ncp, varid, name);
}

int ncmpi_inq_varid(int ncid, const char *name, int *varidp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    return p->driver->inq_varid(p->ncp, name, varidp);
}

static int inq_var_part(int ncid, int varid, char *name, nc_type *xtypep, int *ndimsp, int *dimidsp,
                        int *nattsp, MPI_Offset *offsetp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (varid == NC_GLOBAL) {           /* only ncmpi_inq_varnatts takes NC_GLOBAL (variable.c:463-480) */
        if (nattsp == NULL || name || xtypep || ndimsp || dimidsp || offsetp) return NC_EGLOBAL;
    } else if (varid < 0 || varid >= p->nvars) {
        return NC_ENOTVAR;
    }
    return p->driver->inq_var(p->ncp, varid, name, xtypep, ndimsp, dimidsp, nattsp, offsetp, NULL, NULL);
}

int ncmpi_inq_var(int ncid, int varid, char *name, nc_type *xtypep, int *ndimsp, int *dimidsp, int *nattsp)
{ return inq_var_part(ncid, varid, name, xtypep, ndimsp, dimidsp, nattsp, NULL); }
int ncmpi_inq_varname(int ncid, int varid, char *name)
{ return inq_var_part(ncid, varid, name, NULL, NULL, NULL, NULL, NULL); }
int ncmpi_inq_vartype(int ncid, int varid, nc_type *xtypep)
{ return inq_var_part(ncid, varid, NULL, xtypep, NULL, NULL, NULL, NULL); }
int ncmpi_inq_varndims(int ncid, int varid, int *ndimsp)
{ return inq_var_part(ncid, varid, NULL, NULL, ndimsp, NULL, NULL, NULL); }
int ncmpi_inq_vardimid(int ncid, int varid, int *dimidsp)
{ return inq_var_part(ncid, varid, NULL, NULL, NULL, dimidsp, NULL, NULL); }
int ncmpi_inq_varnatts(int ncid, int varid, int *nattsp)
{ return inq_var_part(ncid, varid, NULL, NULL, NULL, NULL, nattsp, NULL); }
int ncmpi_inq_varoffset(int ncid, int varid, MPI_Offset *offset)
{ return inq_var_part(ncid, varid, NULL, NULL, NULL, NULL, NULL, offset); }

/* ------------------------------------------------------------------------ */
/* attributes (attribute.c, attr_getput.m4)                                  */
/* ------------------------------------------------------------------------ */
static int att_check_get(PNC *p, int varid, const char *name)
{
    if (varid != NC_GLOBAL && (varid < 0 || varid >= p->nvars)) return NC_ENOTVAR;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    return NC_NOERR;
}

static int att_check_put(PNC *p, int varid, const char *name)
{
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;
    return att_check_get(p, varid, name);
}

int ncmpi_inq_att(int ncid, int varid, const char *name, nc_type *xtypep, MPI_Offset *lenp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if ((err = att_check_get(p, varid, name)) != NC_NOERR) return err;
    return p->driver->inq_att(p->ncp, varid, name, xtypep, lenp);
}

int ncmpi_inq_atttype(int ncid, int varid, const char *name, nc_type *xtypep)
{ return ncmpi_inq_att(ncid, varid, name, xtypep, NULL); }
int ncmpi_inq_attlen(int ncid, int varid, const char *name, MPI_Offset *lenp)
{ return ncmpi_inq_att(ncid, varid, name, NULL, lenp); }

int ncmpi_inq_attid(int ncid, int varid, const char *name, int *idp)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if ((err = att_check_get(p, varid, name)) != NC_NOERR) return err;
    return p->driver->inq_attid(p->ncp, varid, name, idp);
}

int ncmpi_inq_attname(int ncid, int varid, int attnum, char *name)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (varid != NC_GLOBAL && (varid < 0 || varid >= p->nvars)) return NC_ENOTVAR;
    return p->driver->inq_attname(p->ncp, varid, attnum, name);
}

int ncmpi_copy_att(int ncid_in, int varid_in, const char *name, int ncid_out, int varid_out)
{
    PNC *pi, *po;
    int err = PNC_check_id(ncid_in, &pi);
    if (err) return err;
    if ((err = PNC_check_id(ncid_out, &po)) != NC_NOERR) return err;
    if (po->flag & NC_MODE_RDONLY) return NC_EPERM;
    if (varid_in != NC_GLOBAL && (varid_in < 0 || varid_in >= pi->nvars)) return NC_ENOTVAR;
    if (varid_out != NC_GLOBAL && (varid_out < 0 || varid_out >= po->nvars)) return NC_ENOTVAR;
    if (name == NULL || *name == 0) return NC_EBADNAME;
    if (strlen(name) > NC_MAX_NAME) return NC_EMAXNAME;
    return pi->driver->copy_att(pi->ncp, varid_in, name, po->ncp, varid_out);
}

int ncmpi_rename_att(int ncid, int varid, const char *name, const char *newname)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if ((err = att_check_put(p, varid, name)) != NC_NOERR) return err;
    if (newname == NULL || *newname == 0) return NC_EBADNAME;
    if (strlen(newname) > NC_MAX_NAME) return NC_EMAXNAME;
    return p->driver->rename_att(p->ncp, varid, name, newname);
}

int ncmpi_del_att(int ncid, int varid, const char *name)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if (p->flag & NC_MODE_RDONLY) return NC_EPERM;
    if (!(p->flag & NC_MODE_DEF)) return NC_ENOTINDEFINE;               /* attribute.c:378-381 */
    if ((err = att_check_get(p, varid, name)) != NC_NOERR) return err;
    return p->driver->del_att(p->ncp, varid, name);
}

/* ncmpii_nc2mpitype (utils.c:25-41) */
static MPI_Datatype nc2mpitype(nc_type t)
{
    switch (t) {
    case NC_BYTE: return MPI_SIGNED_CHAR;
    case NC_CHAR: return MPI_CHAR;
    case NC_SHORT: return MPI_SHORT;
    case NC_INT: return MPI_INT;
    case NC_FLOAT: return MPI_FLOAT;
    case NC_DOUBLE: return MPI_DOUBLE;
    case NC_UBYTE: return MPI_UNSIGNED_CHAR;
    case NC_USHORT: return MPI_UNSIGNED_SHORT;
    case NC_UINT: return MPI_UNSIGNED;
    case NC_INT64: return MPI_LONG_LONG_INT;
    case NC_UINT64: return MPI_UNSIGNED_LONG_LONG;
    default: return MPI_DATATYPE_NULL;
    }
}

/* put_att: sanity_check_put, check_EINVAL, check_EBADTYPE_ECHAR (attr_getput.m4) */
static int put_att(int ncid, int varid, const char *name, nc_type xtype, MPI_Offset nelems, const void *buf,
                   MPI_Datatype itype)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if ((err = att_check_put(p, varid, name)) != NC_NOERR) return err;
    if (nelems > 0 && buf == NULL) return NC_EINVAL;
    if (nelems < 0 || (nelems > NC_MAX_INT && p->format <= NC_FORMAT_CDF2)) return NC_EINVAL;
    if (xtype <= 0 || xtype > NC_UINT64) return NC_EBADTYPE;
    if (p->format <= NC_FORMAT_CDF2 && xtype > NC_DOUBLE) return NC_ESTRICTCDF2;
    if (itype == MPI_DATATYPE_NULL) itype = nc2mpitype(xtype);       /* ncmpi_put_att: buf has xtype's type */
    if ((xtype == NC_CHAR) != (itype == MPI_CHAR)) return NC_ECHAR;
    return p->driver->put_att(p->ncp, varid, name, xtype, nelems, buf, itype);
}

static int get_att(int ncid, int varid, const char *name, void *buf, MPI_Datatype itype)
{
    PNC *p;
    int err = PNC_check_id(ncid, &p);
    if (err) return err;
    if ((err = att_check_get(p, varid, name)) != NC_NOERR) return err;
    if (itype == MPI_DATATYPE_NULL) {             /* ncmpi_get_att: the attribute's own type */
        nc_type xtype;
        if ((err = p->driver->inq_att(p->ncp, varid, name, &xtype, NULL)) != NC_NOERR) return err;
        itype = nc2mpitype(xtype);
    }
    return p->driver->get_att(p->ncp, varid, name, buf, itype);
}

int ncmpi_put_att(int ncid, int varid, const char *name, nc_type xtype, MPI_Offset nelems, const void *value)
{ return put_att(ncid, varid, name, xtype, nelems, value, MPI_DATATYPE_NULL); }
int ncmpi_get_att(int ncid, int varid, const char *name, void *value)
{ return get_att(ncid, varid, name, value, MPI_DATATYPE_NULL); }
int ncmpi_put_att_text(int ncid, int varid, const char *name, MPI_Offset len, const char *op)
{ return put_att(ncid, varid, name, NC_CHAR, len, op, MPI_CHAR); }
int ncmpi_get_att_text(int ncid, int varid, const char *name, char *ip)
{ return get_att(ncid, varid, name, ip, MPI_CHAR); }
int ncmpi_put_att_ubyte(int ncid, int varid, const char *name, nc_type xtype, MPI_Offset len,
                        const unsigned char *op)
{ return put_att(ncid, varid, name, xtype, len, op, MPI_UNSIGNED_CHAR); }
int ncmpi_get_att_ubyte(int ncid, int varid, const char *name, unsigned char *ip)
{ return get_att(ncid, varid, name, ip, MPI_UNSIGNED_CHAR); }

/* the 11 numeric buffer types of the typed APIs, then text (ITYPE_LIST) */
#define PNC_NUM_ITYPES(X)                                             \
    X(schar, signed char, MPI_SIGNED_CHAR)                            \
    X(uchar, unsigned char, MPI_UNSIGNED_CHAR)                        \
    X(short, short, MPI_SHORT)                                        \
    X(ushort, unsigned short, MPI_UNSIGNED_SHORT)                     \
    X(int, int, MPI_INT)                                              \
    X(uint, unsigned int, MPI_UNSIGNED)                               \
    X(long, long, MPI_LONG)                                           \
    X(float, float, MPI_FLOAT)                                        \
    X(double, double, MPI_DOUBLE)                                     \
    X(longlong, long long, MPI_LONG_LONG_INT)                         \
    X(ulonglong, unsigned long long, MPI_UNSIGNED_LONG_LONG)
#define PNC_ITYPES(X) X(text, char, MPI_CHAR) PNC_NUM_ITYPES(X)

#define ATT_API(sfx, ct, mt)                                                                            \
    int ncmpi_put_att_##sfx(int ncid, int varid, const char *name, nc_type xtype, MPI_Offset len,       \
                            const ct *op)                                                               \
    { return put_att(ncid, varid, name, xtype, len, op, mt); }                                          \
    int ncmpi_get_att_##sfx(int ncid, int varid, const char *name, ct *ip)                              \
    { return get_att(ncid, varid, name, ip, mt); }
PNC_NUM_ITYPES(ATT_API)

/* ------------------------------------------------------------------------ */
/* data: argument checks (var_getput.m4:60-284)                              */
/* ------------------------------------------------------------------------ */
typedef enum { API_GET, API_PUT, API_IGET, API_IPUT, API_BPUT } IO_type;

static int check_EINVALCOORDS(int strict, MPI_Offset start, MPI_Offset count, MPI_Offset shape)
{
    if (!strict) {
        if (start < 0 || start > shape) return NC_EINVALCOORDS;
        if (start == shape && count > 0) return NC_EINVALCOORDS;
    } else if (start < 0 || start >= shape) {
        return NC_EINVALCOORDS;
    }
    return NC_NOERR;
}

static int check_EEDGE(const MPI_Offset *start, const MPI_Offset *count, const MPI_Offset *stride,
                       const MPI_Offset *shape)
{
    if (*count > *shape || *start + *count > *shape) return NC_EEDGE;
    if (stride != NULL && *count > 0 && *start + (*count - 1) * (*stride) >= *shape) return NC_EEDGE;
    return NC_NOERR;
}

static int check_start_count_stride(PNC *p, int varid, int isRead, NC_api api, const MPI_Offset *start,
                                    const MPI_Offset *count, const MPI_Offset *stride)
{
    const PNC_var *v = &p->vars[varid];
    const int strict = fIsSet(p->flag, NC_MODE_STRICT_COORD_BOUND);
    MPI_Offset *shape = v->shape;
    int i, err, firstDim = 0;
    if (v->recdim >= 0) {                      /* the current number of records */
        err = p->driver->inq_dim(p->ncp, p->unlimdimid, NULL, &shape[0]);
        if (err) return err;
    }
    if (start == NULL || start[0] < 0) return NC_EINVALCOORDS;
    if (v->recdim >= 0) {
        if ((p->format <= NC_FORMAT_CDF2 || p->format == NC_FORMAT_NETCDF4_CLASSIC) &&
            start[0] > NC_MAX_UINT)
            return NC_EINVALCOORDS;
        if (isRead) {                          /* reads cannot go past numrecs */
            const MPI_Offset len = count == NULL ? 1 : count[0];
            if (shape[0] == 0 && len > 0) return NC_EINVALCOORDS;
            if ((err = check_EINVALCOORDS(strict, start[0], len, shape[0])) != NC_NOERR) return err;
        }
        firstDim = 1;
    }
    for (i = firstDim; i < v->ndims; i++) {
        const MPI_Offset len = count == NULL ? 1 : count[i];
        if ((err = check_EINVALCOORDS(strict, start[i], len, shape[i])) != NC_NOERR) return err;
    }
    if (count == NULL) {
        if (api == API_VARA || api == API_VARS || api == API_VARM) return NC_EEDGE;
        return NC_NOERR;
    }
    firstDim = 0;
    if (v->recdim >= 0) {
        if (count[0] < 0) return NC_ENEGATIVECNT;
        if (isRead && (err = check_EEDGE(start, count, stride, shape)) != NC_NOERR) return err;
        firstDim = 1;
    }
    for (i = firstDim; i < v->ndims; i++) {
        if (shape[i] < 0) return NC_EEDGE;
        if (count[i] < 0) return NC_ENEGATIVECNT;
        err = check_EEDGE(start + i, count + i, stride ? stride + i : NULL, shape + i);
        if (err) return err;
    }
    if (stride != NULL)
        for (i = 0; i < v->ndims; i++)
            if (stride[i] <= 0) return NC_ESTRIDE;
    return NC_NOERR;
}

static int sanity_check(PNC *p, int varid, IO_type io, MPI_Datatype itype, int isColl)
{
    if ((io == API_PUT || io == API_IPUT || io == API_BPUT) && (p->flag & NC_MODE_RDONLY)) return NC_EPERM;
    if (io == API_PUT || io == API_GET) {
        if (p->flag & NC_MODE_DEF) return NC_EINDEFINE;
        if (isColl) {
            if (p->flag & NC_MODE_INDEP) return NC_EINDEP;
        } else if (!(p->flag & NC_MODE_INDEP)) {
            return NC_ENOTINDEP;
        }
    }
    if (varid == NC_GLOBAL) return NC_EGLOBAL;
    if (varid < 0 || varid >= p->nvars) return NC_ENOTVAR;
    if (itype == MPI_DATATYPE_NULL) return NC_NOERR;          /* flexible API */
    if (itype == MPI_CHAR) {
        if (p->vars[varid].xtype != NC_CHAR) return NC_ECHAR;
    } else if (p->vars[varid].xtype == NC_CHAR) {
        return NC_ECHAR;
    }
    return NC_NOERR;
}

static int predefined_buftype(MPI_Datatype t)
{
    return t == MPI_CHAR || t == MPI_SIGNED_CHAR || t == MPI_UNSIGNED_CHAR || t == MPI_SHORT ||
           t == MPI_UNSIGNED_SHORT || t == MPI_INT || t == MPI_UNSIGNED || t == MPI_FLOAT || t == MPI_DOUBLE ||
           t == MPI_LONG_LONG_INT || t == MPI_UNSIGNED_LONG_LONG || t == MPI_LONG;
}

static int allreduce_error(PNC *p, int err)
{
    int minE;
    if (MPI_Allreduce(&err, &minE, 1, MPI_INT, MPI_MIN, p->comm) != MPI_SUCCESS) return NC_EMPI;
    return minE;
}

/* var: the whole variable (GET_FULL_DIMENSIONS); var1: count of ones */
static int full_dims(PNC *p, int varid, MPI_Offset **start, MPI_Offset **count)
{
    const PNC_var *v = &p->vars[varid];
    const int nd = v->ndims;
    int i, err;
    *start = (MPI_Offset *)calloc((size_t)(2 * (nd ? nd : 1)), sizeof(MPI_Offset));
    if (*start == NULL) return NC_ENOMEM;
    *count = *start + (nd ? nd : 1);
    for (i = 0; i < nd; i++) (*count)[i] = v->shape[i];
    if (v->recdim >= 0 && (err = p->driver->inq_dim(p->ncp, p->unlimdimid, NULL, &(*count)[0])) != NC_NOERR) {
        free(*start);
        *start = *count = NULL;
        return err;
    }
    return NC_NOERR;
}

static int ones(PNC *p, int varid, MPI_Offset **count)
{
    const int nd = p->vars[varid].ndims;
    int i;
    *count = (MPI_Offset *)malloc(sizeof(MPI_Offset) * (size_t)(nd ? nd : 1));
    if (*count == NULL) return NC_ENOMEM;
    for (i = 0; i < nd; i++) (*count)[i] = 1;
    return NC_NOERR;
}

/* GETPUT_API (var_getput.m4:330-416): one blocking request */
static int getput(int ncid, int varid, NC_api api, const MPI_Offset *start, const MPI_Offset *count,
                  const MPI_Offset *stride, const MPI_Offset *imap, void *buf, MPI_Offset bufcount,
                  MPI_Datatype buftype, int isRead, int isColl, int hl)
{
    PNC *p;
    int err, status, reqMode = 0;
    MPI_Offset *alloc = NULL, *cnt1 = NULL;
    if ((err = PNC_check_id(ncid, &p)) != NC_NOERR) return err;
    err = sanity_check(p, varid, isRead ? API_GET : API_PUT, hl ? buftype : MPI_DATATYPE_NULL, isColl);
    if (api == API_VARM && imap == NULL) api = stride != NULL ? API_VARS : API_VARA;
    if (api == API_VARS && stride == NULL) api = API_VARA;
    if (!err && api != API_VAR && p->vars[varid].ndims > 0)
        err = check_start_count_stride(p, varid, isRead, api, start, api == API_VAR1 ? NULL : count,
                                       api >= API_VARS ? stride : NULL);
    if (!err && !hl && buftype != MPI_DATATYPE_NULL && bufcount == NC_COUNT_IGNORE && !predefined_buftype(buftype))
        err = NC_EINVAL;
    if (!isColl) {
        if (err) return err;
        if (!hl && buftype != MPI_DATATYPE_NULL && bufcount == 0) return NC_NOERR;
    } else if (p->flag & NC_MODE_SAFE) {
        if ((err = allreduce_error(p, err)) != NC_NOERR) return err;
    } else if (err == NC_EPERM || err == NC_EINDEFINE || err == NC_EINDEP || err == NC_ENOTINDEP) {
        return err;
    } else if (err) {                          /* still take part in the collective */
        int nprocs;
        MPI_Comm_size(p->comm, &nprocs);
        if (nprocs == 1) return err;
        reqMode |= NC_REQ_ZERO;
    }
    reqMode |= (isRead ? NC_REQ_RD : NC_REQ_WR) | NC_REQ_BLK | (hl ? NC_REQ_HL : NC_REQ_FLEX) |
               (isColl ? NC_REQ_COLL : NC_REQ_INDEP);
    if (api == API_VAR && !(reqMode & NC_REQ_ZERO)) {
        int e = full_dims(p, varid, &alloc, &cnt1);
        if (e) { if (!isColl) return e; reqMode |= NC_REQ_ZERO; if (!err) err = e; }
        start = alloc;
        count = cnt1;
    } else if (api == API_VAR1 && !(reqMode & NC_REQ_ZERO)) {
        int e = ones(p, varid, &cnt1);
        if (e) return e;
        count = cnt1;
    }
    if (hl) bufcount = -1;
    if (isRead)
        status = p->driver->get_var(p->ncp, varid, start, count, api >= API_VARS ? stride : NULL,
                                    api == API_VARM ? imap : NULL, buf, bufcount, buftype, reqMode);
    else
        status = p->driver->put_var(p->ncp, varid, start, count, api >= API_VARS ? stride : NULL,
                                    api == API_VARM ? imap : NULL, buf, bufcount, buftype, reqMode);
    if (alloc) free(alloc);
    else free(cnt1);
    return err != NC_NOERR ? err : status;
}

/* IGETPUT_API (var_getput.m4:704-816): one nonblocking request */
static int igetput(int ncid, int varid, NC_api api, const MPI_Offset *start, const MPI_Offset *count,
                   const MPI_Offset *stride, const MPI_Offset *imap, void *buf, MPI_Offset bufcount,
                   MPI_Datatype buftype, IO_type io, int hl, int *reqid)
{
    PNC *p;
    int err, reqMode;
    MPI_Offset *alloc = NULL, *cnt1 = NULL;
    if ((err = PNC_check_id(ncid, &p)) != NC_NOERR) return err;
    if (reqid != NULL) *reqid = NC_REQ_NULL;
    if ((err = sanity_check(p, varid, io, hl ? buftype : MPI_DATATYPE_NULL, 0)) != NC_NOERR) return err;
    if (io == API_BPUT) {                      /* a buffer must be attached */
        MPI_Offset bsize;
        err = p->driver->inq_misc(p->ncp, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL,
                                  NULL, NULL, &bsize);
        if (err) return err;
    }
    if (api == API_VARM && imap == NULL) api = stride != NULL ? API_VARS : API_VARA;
    if (api == API_VARS && stride == NULL) api = API_VARA;
    if (api != API_VAR && p->vars[varid].ndims > 0) {
        err = check_start_count_stride(p, varid, io == API_IGET, api, start, api == API_VAR1 ? NULL : count,
                                       api >= API_VARS ? stride : NULL);
        if (err) return err;
    }
    if (!hl && buftype != MPI_DATATYPE_NULL && bufcount == 0) return NC_NOERR;
    if (!hl && buftype != MPI_DATATYPE_NULL && bufcount == NC_COUNT_IGNORE && !predefined_buftype(buftype))
        return NC_EINVAL;
    reqMode = (io == API_IGET ? NC_REQ_RD : NC_REQ_WR) | (io == API_BPUT ? NC_REQ_NBB : NC_REQ_NBI) |
              (hl ? NC_REQ_HL : NC_REQ_FLEX);
    if (api == API_VAR) {
        if ((err = full_dims(p, varid, &alloc, &cnt1)) != NC_NOERR) return err;
        start = alloc;
        count = cnt1;
    } else if (api == API_VAR1) {
        if ((err = ones(p, varid, &cnt1)) != NC_NOERR) return err;
        count = cnt1;
    }
    if (hl) bufcount = -1;
    stride = api >= API_VARS ? stride : NULL;
    imap = api == API_VARM ? imap : NULL;
    if (io == API_IGET)
        err = p->driver->iget_var(p->ncp, varid, start, count, stride, imap, buf, bufcount, buftype, reqid, reqMode);
    else if (io == API_IPUT)
        err = p->driver->iput_var(p->ncp, varid, start, count, stride, imap, buf, bufcount, buftype, reqid, reqMode);
    else
        err = p->driver->bput_var(p->ncp, varid, start, count, stride, imap, buf, bufcount, buftype, reqid, reqMode);
    if (alloc) free(alloc);
    else free(cnt1);
    return err;
}

/* starts/counts of a varn: checked box by box (var_getput.m4:466-497) */
static int check_varn(PNC *p, int varid, int isRead, int num, MPI_Offset *const *starts,
                      MPI_Offset *const *counts)
{
    int i, err;
    if (starts == NULL) return NC_ENULLSTART;
    for (i = 0; i < num; i++) {
        const int one = counts == NULL || counts[i] == NULL;
        if (starts[i] == NULL) return NC_ENULLSTART;
        err = check_start_count_stride(p, varid, isRead, one ? API_VAR1 : API_VARA, starts[i],
                                       one ? NULL : counts[i], NULL);
        if (err) return err;
    }
    return NC_NOERR;
}

/* VARN (var_getput.m4:436-529) */
static int varn(int ncid, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts, void *buf,
                MPI_Offset bufcount, MPI_Datatype buftype, int isRead, int isColl, int hl)
{
    PNC *p;
    int err, status, reqMode = 0, isScalar = 0;
    if ((err = PNC_check_id(ncid, &p)) != NC_NOERR) return err;
    err = sanity_check(p, varid, isRead ? API_GET : API_PUT, hl ? buftype : MPI_DATATYPE_NULL, isColl);
    if (!err && num != 0) {
        if (p->vars[varid].ndims == 0) {
            isScalar = 1;
            if (num != 1) err = NC_EINVAL;
        } else {
            err = check_varn(p, varid, isRead, num, starts, counts);
        }
    }
    if (!err && num != 0 && !hl && buftype != MPI_DATATYPE_NULL && bufcount == NC_COUNT_IGNORE &&
        !predefined_buftype(buftype))
        err = NC_EINVAL;
    if (!isColl) {
        if (err) return err;
        if (num == 0) return NC_NOERR;
    } else if (p->flag & NC_MODE_SAFE) {
        if ((err = allreduce_error(p, err)) != NC_NOERR) return err;
    } else if (err == NC_EPERM || err == NC_EINDEFINE || err == NC_EINDEP || err == NC_ENOTINDEP) {
        return err;
    } else if (err) {
        int nprocs;
        MPI_Comm_size(p->comm, &nprocs);
        if (nprocs == 1) return err;
        reqMode |= NC_REQ_ZERO;
    } else if (num == 0) {
        reqMode |= NC_REQ_ZERO;
    }
    reqMode |= (isRead ? NC_REQ_RD : NC_REQ_WR) | NC_REQ_BLK | (hl ? NC_REQ_HL : NC_REQ_FLEX) |
               (isColl ? NC_REQ_COLL : NC_REQ_INDEP);
    if (hl) bufcount = -1;
    if (isScalar) {
        MPI_Offset s0[1] = {0}, c0[1] = {1};
        status = isRead ? p->driver->get_var(p->ncp, varid, s0, c0, NULL, NULL, buf, bufcount, buftype, reqMode)
                        : p->driver->put_var(p->ncp, varid, s0, c0, NULL, NULL, buf, bufcount, buftype, reqMode);
    } else {
        status = isRead ? p->driver->get_varn(p->ncp, varid, num, starts, counts, buf, bufcount, buftype, reqMode)
                        : p->driver->put_varn(p->ncp, varid, num, starts, counts, buf, bufcount, buftype, reqMode);
    }
    return err != NC_NOERR ? err : status;
}

/* IVARN (var_getput.m4:830-940) */
static int ivarn(int ncid, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts, void *buf,
                 MPI_Offset bufcount, MPI_Datatype buftype, IO_type io, int hl, int *reqid)
{
    PNC *p;
    int err, reqMode;
    if ((err = PNC_check_id(ncid, &p)) != NC_NOERR) return err;
    if (reqid != NULL) *reqid = NC_REQ_NULL;
    if ((err = sanity_check(p, varid, io, hl ? buftype : MPI_DATATYPE_NULL, 0)) != NC_NOERR) return err;
    if (num == 0) return NC_NOERR;
    if (io == API_BPUT) {
        MPI_Offset bsize;
        err = p->driver->inq_misc(p->ncp, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL,
                                  NULL, NULL, &bsize);
        if (err) return err;
    }
    if (!hl && buftype != MPI_DATATYPE_NULL && bufcount == 0) return NC_NOERR;
    if (!hl && buftype != MPI_DATATYPE_NULL && bufcount == NC_COUNT_IGNORE && !predefined_buftype(buftype))
        return NC_EINVAL;
    reqMode = (io == API_IGET ? NC_REQ_RD : NC_REQ_WR) | (io == API_BPUT ? NC_REQ_NBB : NC_REQ_NBI) |
              (hl ? NC_REQ_HL : NC_REQ_FLEX);
    if (hl) bufcount = -1;
    if (p->vars[varid].ndims == 0) {
        MPI_Offset s0[1] = {0}, c0[1] = {1};
        if (num != 1) return NC_EINVAL;
        if (io == API_IGET)
            return p->driver->iget_var(p->ncp, varid, s0, c0, NULL, NULL, buf, bufcount, buftype, reqid, reqMode);
        if (io == API_IPUT)
            return p->driver->iput_var(p->ncp, varid, s0, c0, NULL, NULL, buf, bufcount, buftype, reqid, reqMode);
        return p->driver->bput_var(p->ncp, varid, s0, c0, NULL, NULL, buf, bufcount, buftype, reqid, reqMode);
    }
    if ((err = check_varn(p, varid, io == API_IGET, num, starts, counts)) != NC_NOERR) return err;
    if (io == API_IGET)
        return p->driver->iget_varn(p->ncp, varid, num, starts, counts, buf, bufcount, buftype, reqid, reqMode);
    if (io == API_IPUT)
        return p->driver->iput_varn(p->ncp, varid, num, starts, counts, buf, bufcount, buftype, reqid, reqMode);
    return p->driver->bput_varn(p->ncp, varid, num, starts, counts, buf, bufcount, buftype, reqid, reqMode);
}

/* MVAR (var_getput.m4:560-700): one nonblocking request per variable, then
 * one wait.  bufcounts/buftypes NULL: the typed form (buftype `mt`). */
static int mvar(int ncid, int nvars, int *varids, NC_api api, MPI_Offset *const *starts, MPI_Offset *const *counts,
                MPI_Offset *const *strides, MPI_Offset *const *imaps, void *const *bufs, const MPI_Offset *bufcounts,
                const MPI_Datatype *buftypes, MPI_Datatype mt, int isRead, int isColl)
{
    PNC *p;
    int i, err = NC_NOERR, status, reqMode, *reqs;
    const int hl = buftypes == NULL;
    if ((err = PNC_check_id(ncid, &p)) != NC_NOERR) return err;
    if (!isColl && nvars == 0) return NC_NOERR;
    if (api == API_VARM && imaps == NULL) api = strides != NULL ? API_VARS : API_VARA;
    if (api == API_VARS && strides == NULL) api = API_VARA;
    for (i = 0; i < nvars; i++) {
        err = sanity_check(p, varids[i], isRead ? API_GET : API_PUT, hl ? mt : MPI_DATATYPE_NULL, isColl);
        if (err) break;
        if (api != API_VAR && p->vars[varids[i]].ndims > 0) {
            err = check_start_count_stride(p, varids[i], isRead, api, starts[i],
                                           api == API_VAR1 ? NULL : counts[i],
                                           (api >= API_VARS && strides) ? strides[i] : NULL);
            if (err) break;
        }
        if (!hl && buftypes[i] != MPI_DATATYPE_NULL && bufcounts[i] == NC_COUNT_IGNORE &&
            !predefined_buftype(buftypes[i])) {
            err = NC_EINVAL;
            break;
        }
    }
    reqMode = (isRead ? NC_REQ_RD : NC_REQ_WR) | NC_REQ_NBI | (hl ? NC_REQ_HL : NC_REQ_FLEX) |
              (isColl ? NC_REQ_COLL : NC_REQ_INDEP);
    if (!isColl) {
        if (err) return err;
    } else if (p->flag & NC_MODE_SAFE) {
        if ((err = allreduce_error(p, err)) != NC_NOERR) return err;
    } else if (err == NC_EPERM || err == NC_EINDEFINE || err == NC_EINDEP || err == NC_ENOTINDEP) {
        return err;
    } else if (err) {
        p->driver->wait(p->ncp, 0, NULL, NULL, reqMode);   /* take part in the collective */
        return err;
    }
    reqs = (int *)malloc(sizeof(int) * (size_t)(nvars > 0 ? nvars : 1));
    if (reqs == NULL) return NC_ENOMEM;
    for (i = 0; i < nvars; i++) {
        MPI_Offset *alloc = NULL, *cnt1 = NULL;
        const MPI_Offset *start = NULL, *count = NULL, *stride = NULL, *imap = NULL;
        if (api == API_VAR) {
            if ((err = full_dims(p, varids[i], &alloc, &cnt1)) != NC_NOERR) break;
            start = alloc;
            count = cnt1;
        } else if (api == API_VAR1) {
            if ((err = ones(p, varids[i], &cnt1)) != NC_NOERR) break;
            start = starts[i];
            count = cnt1;
        } else {
            start = starts[i];
            count = counts[i];
        }
        if (api >= API_VARS && strides) stride = strides[i];
        if (api == API_VARM && imaps) imap = imaps[i];
        if (isRead)
            err = p->driver->iget_var(p->ncp, varids[i], start, count, stride, imap, bufs[i],
                                      hl ? -1 : bufcounts[i], hl ? mt : buftypes[i], &reqs[i], reqMode);
        else
            err = p->driver->iput_var(p->ncp, varids[i], start, count, stride, imap, bufs[i],
                                      hl ? -1 : bufcounts[i], hl ? mt : buftypes[i], &reqs[i], reqMode);
        if (alloc) free(alloc);
        else free(cnt1);
        if (err) break;
    }
    status = p->driver->wait(p->ncp, i, reqs, NULL, reqMode);
    free(reqs);
    return err != NC_NOERR ? err : status;
}

/* ------------------------------------------------------------------------ */
/* data: the entry points                                                    */
/* ------------------------------------------------------------------------ */
#define BUF_FLEX_PUT const void *op, MPI_Offset bufcount, MPI_Datatype buftype
#define BUF_FLEX_GET void *ip, MPI_Offset bufcount, MPI_Datatype buftype
#define A_START const MPI_Offset *start
#define A_COUNT const MPI_Offset *count
#define A_STRIDE const MPI_Offset *stride
#define A_IMAP const MPI_Offset *imap

/* flexible blocking (buftype given) */
#define FLEX_BLOCKING(coll, isColl)                                                                             \
    int ncmpi_put_var##coll(int ncid, int varid, BUF_FLEX_PUT)                                                  \
    { return getput(ncid, varid, API_VAR, NULL, NULL, NULL, NULL, (void *)op, bufcount, buftype, 0, isColl, 0); } \
    int ncmpi_get_var##coll(int ncid, int varid, BUF_FLEX_GET)                                                  \
    { return getput(ncid, varid, API_VAR, NULL, NULL, NULL, NULL, ip, bufcount, buftype, 1, isColl, 0); }        \
    int ncmpi_put_var1##coll(int ncid, int varid, A_START, BUF_FLEX_PUT)                                        \
    { return getput(ncid, varid, API_VAR1, start, NULL, NULL, NULL, (void *)op, bufcount, buftype, 0, isColl, 0); } \
    int ncmpi_get_var1##coll(int ncid, int varid, A_START, BUF_FLEX_GET)                                        \
    { return getput(ncid, varid, API_VAR1, start, NULL, NULL, NULL, ip, bufcount, buftype, 1, isColl, 0); }      \
    int ncmpi_put_vara##coll(int ncid, int varid, A_START, A_COUNT, BUF_FLEX_PUT)                               \
    { return getput(ncid, varid, API_VARA, start, count, NULL, NULL, (void *)op, bufcount, buftype, 0, isColl, 0); } \
    int ncmpi_get_vara##coll(int ncid, int varid, A_START, A_COUNT, BUF_FLEX_GET)                               \
    { return getput(ncid, varid, API_VARA, start, count, NULL, NULL, ip, bufcount, buftype, 1, isColl, 0); }     \
    int ncmpi_put_vars##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, BUF_FLEX_PUT)                     \
    { return getput(ncid, varid, API_VARS, start, count, stride, NULL, (void *)op, bufcount, buftype, 0, isColl, 0); } \
    int ncmpi_get_vars##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, BUF_FLEX_GET)                     \
    { return getput(ncid, varid, API_VARS, start, count, stride, NULL, ip, bufcount, buftype, 1, isColl, 0); }   \
    int ncmpi_put_varm##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, A_IMAP, BUF_FLEX_PUT)             \
    { return getput(ncid, varid, API_VARM, start, count, stride, imap, (void *)op, bufcount, buftype, 0, isColl, 0); } \
    int ncmpi_get_varm##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, A_IMAP, BUF_FLEX_GET)             \
    { return getput(ncid, varid, API_VARM, start, count, stride, imap, ip, bufcount, buftype, 1, isColl, 0); }   \
    int ncmpi_put_varn##coll(int ncid, int varid, int num, MPI_Offset *const *starts,                           \
                             MPI_Offset *const *counts, BUF_FLEX_PUT)                                           \
    { return varn(ncid, varid, num, starts, counts, (void *)op, bufcount, buftype, 0, isColl, 0); }             \
    int ncmpi_get_varn##coll(int ncid, int varid, int num, MPI_Offset *const *starts,                           \
                             MPI_Offset *const *counts, BUF_FLEX_GET)                                           \
    { return varn(ncid, varid, num, starts, counts, ip, bufcount, buftype, 1, isColl, 0); }
FLEX_BLOCKING(, 0)
FLEX_BLOCKING(_all, 1)

/* typed blocking: ncmpi_{put,get}_var{,1,a,s,m,n}_<type>[_all] */
#define TYPED_BLOCKING_C(sfx, ct, mt, coll, isColl)                                                             \
    int ncmpi_put_var_##sfx##coll(int ncid, int varid, const ct *op)                                            \
    { return getput(ncid, varid, API_VAR, NULL, NULL, NULL, NULL, (void *)op, -1, mt, 0, isColl, 1); }          \
    int ncmpi_get_var_##sfx##coll(int ncid, int varid, ct *ip)                                                  \
    { return getput(ncid, varid, API_VAR, NULL, NULL, NULL, NULL, ip, -1, mt, 1, isColl, 1); }                  \
    int ncmpi_put_var1_##sfx##coll(int ncid, int varid, A_START, const ct *op)                                  \
    { return getput(ncid, varid, API_VAR1, start, NULL, NULL, NULL, (void *)op, -1, mt, 0, isColl, 1); }        \
    int ncmpi_get_var1_##sfx##coll(int ncid, int varid, A_START, ct *ip)                                        \
    { return getput(ncid, varid, API_VAR1, start, NULL, NULL, NULL, ip, -1, mt, 1, isColl, 1); }                \
    int ncmpi_put_vara_##sfx##coll(int ncid, int varid, A_START, A_COUNT, const ct *op)                         \
    { return getput(ncid, varid, API_VARA, start, count, NULL, NULL, (void *)op, -1, mt, 0, isColl, 1); }       \
    int ncmpi_get_vara_##sfx##coll(int ncid, int varid, A_START, A_COUNT, ct *ip)                               \
    { return getput(ncid, varid, API_VARA, start, count, NULL, NULL, ip, -1, mt, 1, isColl, 1); }               \
    int ncmpi_put_vars_##sfx##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, const ct *op)               \
    { return getput(ncid, varid, API_VARS, start, count, stride, NULL, (void *)op, -1, mt, 0, isColl, 1); }     \
    int ncmpi_get_vars_##sfx##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, ct *ip)                     \
    { return getput(ncid, varid, API_VARS, start, count, stride, NULL, ip, -1, mt, 1, isColl, 1); }             \
    int ncmpi_put_varm_##sfx##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, A_IMAP, const ct *op)       \
    { return getput(ncid, varid, API_VARM, start, count, stride, imap, (void *)op, -1, mt, 0, isColl, 1); }     \
    int ncmpi_get_varm_##sfx##coll(int ncid, int varid, A_START, A_COUNT, A_STRIDE, A_IMAP, ct *ip)             \
    { return getput(ncid, varid, API_VARM, start, count, stride, imap, ip, -1, mt, 1, isColl, 1); }             \
    int ncmpi_put_varn_##sfx##coll(int ncid, int varid, int num, MPI_Offset *const *starts,                     \
                                   MPI_Offset *const *counts, const ct *op)                                     \
    { return varn(ncid, varid, num, starts, counts, (void *)op, -1, mt, 0, isColl, 1); }                        \
    int ncmpi_get_varn_##sfx##coll(int ncid, int varid, int num, MPI_Offset *const *starts,                     \
                                   MPI_Offset *const *counts, ct *ip)                                           \
    { return varn(ncid, varid, num, starts, counts, ip, -1, mt, 1, isColl, 1); }
#define TYPED_BLOCKING(sfx, ct, mt) TYPED_BLOCKING_C(sfx, ct, mt, , 0) TYPED_BLOCKING_C(sfx, ct, mt, _all, 1)
PNC_ITYPES(TYPED_BLOCKING)

/* flexible nonblocking: ncmpi_{iput,iget,bput}_var{,1,a,s,m,n} */
#define FLEX_NB(op_, io, CONST)                                                                                 \
    int ncmpi_##op_##_var(int ncid, int varid, CONST void *buf, MPI_Offset bufcount, MPI_Datatype buftype,     \
                          int *req)                                                                             \
    { return igetput(ncid, varid, API_VAR, NULL, NULL, NULL, NULL, (void *)buf, bufcount, buftype, io, 0, req); } \
    int ncmpi_##op_##_var1(int ncid, int varid, A_START, CONST void *buf, MPI_Offset bufcount,                 \
                           MPI_Datatype buftype, int *req)                                                      \
    { return igetput(ncid, varid, API_VAR1, start, NULL, NULL, NULL, (void *)buf, bufcount, buftype, io, 0, req); } \
    int ncmpi_##op_##_vara(int ncid, int varid, A_START, A_COUNT, CONST void *buf, MPI_Offset bufcount,        \
                           MPI_Datatype buftype, int *req)                                                      \
    { return igetput(ncid, varid, API_VARA, start, count, NULL, NULL, (void *)buf, bufcount, buftype, io, 0, req); } \
    int ncmpi_##op_##_vars(int ncid, int varid, A_START, A_COUNT, A_STRIDE, CONST void *buf,                   \
                           MPI_Offset bufcount, MPI_Datatype buftype, int *req)                                 \
    { return igetput(ncid, varid, API_VARS, start, count, stride, NULL, (void *)buf, bufcount, buftype, io, 0,  \
                     req); }                                                                                    \
    int ncmpi_##op_##_varm(int ncid, int varid, A_START, A_COUNT, A_STRIDE, A_IMAP, CONST void *buf,           \
                           MPI_Offset bufcount, MPI_Datatype buftype, int *req)                                 \
    { return igetput(ncid, varid, API_VARM, start, count, stride, imap, (void *)buf, bufcount, buftype, io, 0,  \
                     req); }                                                                                    \
    int ncmpi_##op_##_varn(int ncid, int varid, int num, MPI_Offset *const *starts, MPI_Offset *const *counts, \
                           CONST void *buf, MPI_Offset bufcount, MPI_Datatype buftype, int *req)                \
    { return ivarn(ncid, varid, num, starts, counts, (void *)buf, bufcount, buftype, io, 0, req); }
#define NOCONST
FLEX_NB(iput, API_IPUT, const)
FLEX_NB(iget, API_IGET, NOCONST)
FLEX_NB(bput, API_BPUT, const)

/* typed nonblocking: ncmpi_{iput,iget,bput}_var{,1,a,s,m,n}_<type> */
#define TYPED_NB_OP(sfx, ct, mt, op_, io, CONST)                                                                \
    int ncmpi_##op_##_var_##sfx(int ncid, int varid, CONST ct *buf, int *req)                                  \
    { return igetput(ncid, varid, API_VAR, NULL, NULL, NULL, NULL, (void *)buf, -1, mt, io, 1, req); }          \
    int ncmpi_##op_##_var1_##sfx(int ncid, int varid, A_START, CONST ct *buf, int *req)                        \
    { return igetput(ncid, varid, API_VAR1, start, NULL, NULL, NULL, (void *)buf, -1, mt, io, 1, req); }        \
    int ncmpi_##op_##_vara_##sfx(int ncid, int varid, A_START, A_COUNT, CONST ct *buf, int *req)               \
    { return igetput(ncid, varid, API_VARA, start, count, NULL, NULL, (void *)buf, -1, mt, io, 1, req); }       \
    int ncmpi_##op_##_vars_##sfx(int ncid, int varid, A_START, A_COUNT, A_STRIDE, CONST ct *buf, int *req)     \
    { return igetput(ncid, varid, API_VARS, start, count, stride, NULL, (void *)buf, -1, mt, io, 1, req); }     \
    int ncmpi_##op_##_varm_##sfx(int ncid, int varid, A_START, A_COUNT, A_STRIDE, A_IMAP, CONST ct *buf,       \
                                 int *req)                                                                      \
    { return igetput(ncid, varid, API_VARM, start, count, stride, imap, (void *)buf, -1, mt, io, 1, req); }     \
    int ncmpi_##op_##_varn_##sfx(int ncid, int varid, int num, MPI_Offset *const *starts,                      \
                                 MPI_Offset *const *counts, CONST ct *buf, int *req)                            \
    { return ivarn(ncid, varid, num, starts, counts, (void *)buf, -1, mt, io, 1, req); }
#define TYPED_NB(sfx, ct, mt)                          \
    TYPED_NB_OP(sfx, ct, mt, iput, API_IPUT, const)    \
    TYPED_NB_OP(sfx, ct, mt, iget, API_IGET, NOCONST)  \
    TYPED_NB_OP(sfx, ct, mt, bput, API_BPUT, const)
PNC_ITYPES(TYPED_NB)

/* multi-variable: ncmpi_{mput,mget}_var{,1,a,s,m}[_<type>][_all] */
#define M_STARTS MPI_Offset *const *starts
#define M_COUNTS MPI_Offset *const *counts
#define M_STRIDES MPI_Offset *const *strides
#define M_IMAPS MPI_Offset *const *imaps
#define FLEX_M(coll, isColl)                                                                                    \
    int ncmpi_mput_var##coll(int ncid, int num, int *varids, void *const *buf, const MPI_Offset *bufcounts,     \
                             const MPI_Datatype datatypes[])                                                    \
    { return mvar(ncid, num, varids, API_VAR, NULL, NULL, NULL, NULL, buf, bufcounts, datatypes,               \
                  MPI_DATATYPE_NULL, 0, isColl); }                                                              \
    int ncmpi_mget_var##coll(int ncid, int num, int *varids, void *bufs[], const MPI_Offset *bufcounts,        \
                             const MPI_Datatype *datatypes)                                                     \
    { return mvar(ncid, num, varids, API_VAR, NULL, NULL, NULL, NULL, bufs, bufcounts, datatypes,              \
                  MPI_DATATYPE_NULL, 1, isColl); }                                                              \
    int ncmpi_mput_var1##coll(int ncid, int num, int *varids, M_STARTS, void *const *buf,                      \
                              const MPI_Offset *bufcounts, const MPI_Datatype datatypes[])                      \
    { return mvar(ncid, num, varids, API_VAR1, starts, NULL, NULL, NULL, buf, bufcounts, datatypes,            \
                  MPI_DATATYPE_NULL, 0, isColl); }                                                              \
    int ncmpi_mget_var1##coll(int ncid, int num, int *varids, M_STARTS, void *bufs[],                          \
                              const MPI_Offset *bufcounts, const MPI_Datatype *datatypes)                       \
    { return mvar(ncid, num, varids, API_VAR1, starts, NULL, NULL, NULL, bufs, bufcounts, datatypes,           \
                  MPI_DATATYPE_NULL, 1, isColl); }                                                              \
    int ncmpi_mput_vara##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, void *const *buf,            \
                              const MPI_Offset *bufcounts, const MPI_Datatype datatypes[])                      \
    { return mvar(ncid, num, varids, API_VARA, starts, counts, NULL, NULL, buf, bufcounts, datatypes,          \
                  MPI_DATATYPE_NULL, 0, isColl); }                                                              \
    int ncmpi_mget_vara##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, void *bufs[],                \
                              const MPI_Offset *bufcounts, const MPI_Datatype *datatypes)                       \
    { return mvar(ncid, num, varids, API_VARA, starts, counts, NULL, NULL, bufs, bufcounts, datatypes,         \
                  MPI_DATATYPE_NULL, 1, isColl); }                                                              \
    int ncmpi_mput_vars##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES, void *const *buf, \
                              const MPI_Offset *bufcounts, const MPI_Datatype datatypes[])                      \
    { return mvar(ncid, num, varids, API_VARS, starts, counts, strides, NULL, buf, bufcounts, datatypes,       \
                  MPI_DATATYPE_NULL, 0, isColl); }                                                              \
    int ncmpi_mget_vars##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES, void *bufs[],     \
                              const MPI_Offset *bufcounts, const MPI_Datatype *datatypes)                       \
    { return mvar(ncid, num, varids, API_VARS, starts, counts, strides, NULL, bufs, bufcounts, datatypes,      \
                  MPI_DATATYPE_NULL, 1, isColl); }                                                              \
    int ncmpi_mput_varm##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES, M_IMAPS,          \
                              void *const *buf, const MPI_Offset *bufcounts, const MPI_Datatype datatypes[])    \
    { return mvar(ncid, num, varids, API_VARM, starts, counts, strides, imaps, buf, bufcounts, datatypes,      \
                  MPI_DATATYPE_NULL, 0, isColl); }                                                              \
    int ncmpi_mget_varm##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES, M_IMAPS,          \
                              void *bufs[], const MPI_Offset *bufcounts, const MPI_Datatype *datatypes)         \
    { return mvar(ncid, num, varids, API_VARM, starts, counts, strides, imaps, bufs, bufcounts, datatypes,     \
                  MPI_DATATYPE_NULL, 1, isColl); }
FLEX_M(, 0)
FLEX_M(_all, 1)

#define TYPED_M_C(sfx, ct, mt, coll, isColl)                                                                    \
    int ncmpi_mput_var_##sfx##coll(int ncid, int num, int *varids, ct *const *buf)                             \
    { return mvar(ncid, num, varids, API_VAR, NULL, NULL, NULL, NULL, (void *const *)buf, NULL, NULL, mt, 0,   \
                  isColl); }                                                                                    \
    int ncmpi_mget_var_##sfx##coll(int ncid, int num, int *varids, ct *bufs[])                                 \
    { return mvar(ncid, num, varids, API_VAR, NULL, NULL, NULL, NULL, (void *const *)bufs, NULL, NULL, mt, 1,  \
                  isColl); }                                                                                    \
    int ncmpi_mput_var1_##sfx##coll(int ncid, int num, int *varids, M_STARTS, ct *const *buf)                  \
    { return mvar(ncid, num, varids, API_VAR1, starts, NULL, NULL, NULL, (void *const *)buf, NULL, NULL, mt, 0, \
                  isColl); }                                                                                    \
    int ncmpi_mget_var1_##sfx##coll(int ncid, int num, int *varids, M_STARTS, ct *bufs[])                      \
    { return mvar(ncid, num, varids, API_VAR1, starts, NULL, NULL, NULL, (void *const *)bufs, NULL, NULL, mt,  \
                  1, isColl); }                                                                                 \
    int ncmpi_mput_vara_##sfx##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, ct *const *buf)        \
    { return mvar(ncid, num, varids, API_VARA, starts, counts, NULL, NULL, (void *const *)buf, NULL, NULL, mt,  \
                  0, isColl); }                                                                                 \
    int ncmpi_mget_vara_##sfx##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, ct *bufs[])            \
    { return mvar(ncid, num, varids, API_VARA, starts, counts, NULL, NULL, (void *const *)bufs, NULL, NULL, mt, \
                  1, isColl); }                                                                                 \
    int ncmpi_mput_vars_##sfx##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES,             \
                                    ct *const *buf)                                                             \
    { return mvar(ncid, num, varids, API_VARS, starts, counts, strides, NULL, (void *const *)buf, NULL, NULL,  \
                  mt, 0, isColl); }                                                                             \
    int ncmpi_mget_vars_##sfx##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES,             \
                                    ct *bufs[])                                                                 \
    { return mvar(ncid, num, varids, API_VARS, starts, counts, strides, NULL, (void *const *)bufs, NULL, NULL, \
                  mt, 1, isColl); }                                                                             \
    int ncmpi_mput_varm_##sfx##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES, M_IMAPS,    \
                                    ct *const *buf)                                                             \
    { return mvar(ncid, num, varids, API_VARM, starts, counts, strides, imaps, (void *const *)buf, NULL, NULL, \
                  mt, 0, isColl); }                                                                             \
    int ncmpi_mget_varm_##sfx##coll(int ncid, int num, int *varids, M_STARTS, M_COUNTS, M_STRIDES, M_IMAPS,    \
                                    ct *bufs[])                                                                 \
    { return mvar(ncid, num, varids, API_VARM, starts, counts, strides, imaps, (void *const *)bufs, NULL,      \
                  NULL, mt, 1, isColl); }
#define TYPED_M(sfx, ct, mt) TYPED_M_C(sfx, ct, mt, , 0) TYPED_M_C(sfx, ct, mt, _all, 1)
PNC_ITYPES(TYPED_M)

/* vard: deprecated by the reference in 1.15.0 (var_getput.m4:950-970) */
#define VARD(op_, CONST, coll)                                                                                  \
    int ncmpi_##op_##_vard##coll(int ncid, int varid, MPI_Datatype filetype, CONST void *buf,                  \
                                 MPI_Offset bufcount, MPI_Datatype buftype)                                     \
    {                                                                                                           \
        (void)ncid; (void)varid; (void)filetype; (void)buf; (void)bufcount; (void)buftype;                      \
        fprintf(stderr, "PnetCDF vard APIs have been deprecated since 1.15.0 release.\n");                     \
        return NC_ENOTSUPPORT;                                                                                  \
    }
VARD(put, const, )
VARD(put, const, _all)
VARD(get, NOCONST, )
VARD(get, NOCONST, _all)
