"""Generate include/pnetcdf.h: the public ncmpi_* C API of PnetCDF 1.15.0 as
this library exports it (libpnetcdf.so), so programs written against the
reference (e.g. benchmarks/C/pnetcdf_put_vara.c) compile unchanged.

The reference generates its header from src/include/pnetcdf.h.in with m4
(ITYPE_LIST = text schar uchar short ushort int uint long float double
longlong ulonglong); the same families are produced here from one table:
  blocking     ncmpi_{put,get}_var{,1,a,s,m}[_<type>][_all]   pnetcdf.h.in:1100-2330
  varn         ncmpi_{put,get}_varn[_<type>][_all]            :2080-2330
  vard         ncmpi_{put,get}_vard[_all]                     :2326-2340
  nonblocking  ncmpi_{iput,iget,bput}_var{,1,a,s,m,n}[_<type>]:2369-3470
  multi-var    ncmpi_{mput,mget}_var{,1,a,s,m}[_<type>][_all] :3480-4560
Constants and the non-data prototypes are restated from pnetcdf.h.in:66-930
(values are the public ABI; NC_* spellings match include/pncx.h and
include/pncx_nc.h token for token, so the headers can be included together).

    python tools/gen_pnetcdf_h.py          (rewrites include/pnetcdf.h)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TYPES = [("text", "char"), ("schar", "signed char"), ("uchar", "unsigned char"), ("short", "short"),
         ("ushort", "unsigned short"), ("int", "int"), ("uint", "unsigned int"), ("long", "long"),
         ("float", "float"), ("double", "double"), ("longlong", "long long"),
         ("ulonglong", "unsigned long long")]

KIND_ARGS = {"": "", "1": ", const MPI_Offset *start",
             "a": ", const MPI_Offset *start, const MPI_Offset *count",
             "s": ", const MPI_Offset *start, const MPI_Offset *count, const MPI_Offset *stride",
             "m": ", const MPI_Offset *start, const MPI_Offset *count, const MPI_Offset *stride, "
                  "const MPI_Offset *imap"}
MKIND_ARGS = {"": "", "1": ", MPI_Offset* const *starts",
              "a": ", MPI_Offset* const *starts, MPI_Offset* const *counts",
              "s": ", MPI_Offset* const *starts, MPI_Offset* const *counts, MPI_Offset* const *strides",
              "m": ", MPI_Offset* const *starts, MPI_Offset* const *counts, MPI_Offset* const *strides, "
                   "MPI_Offset* const *imaps"}
VARN_ARGS = ", int num, MPI_Offset* const *starts, MPI_Offset* const *counts"

CONSTANTS = r'''
#define PNETCDF_VERSION       "1.15.0"
#define PNETCDF_VERSION_MAJOR 1
#define PNETCDF_VERSION_MINOR 15
#define PNETCDF_VERSION_SUB   0
#define PNETCDF_VERSION_PRE   ""
#define PNETCDF_RELEASE_DATE  "MI355X"

/* features of this build (pnetcdf.h.in:25-40); conversion runs on the GPU */
#define PNETCDF_ENABLE_FORTRAN           0
#define PNETCDF_ENABLE_CXX               0
#define PNETCDF_ERANGE_FILL              1
#define PNETCDF_SUBFILING                0
#define PNETCDF_RELAX_COORD_BOUND        1
#define PNETCDF_DEBUG_MODE               0
#define PNETCDF_PROFILING                0
#define PNETCDF_NULL_BYTE_HEADER_PADDING 0
#define PNETCDF_BYTE_SWAP_IN_PLACE       0
#define PNETCDF_BURST_BUFFERING          0
#define PNETCDF_THREAD_SAFE              0
#define PNETCDF_DRIVER_NETCDF4           0
#define PNETCDF_DRIVER_ADIOS             0
#define PNETCDF_DRIVER_GIO               0
#define PNETCDF_DRIVER_MI355X            1

#ifndef _NETCDF_
typedef int nc_type;

/* external data types (pnetcdf.h.in:66-83) */
#define NC_NAT     0
#define NC_BYTE    1
#define NC_CHAR    2
#define NC_SHORT   3
#define NC_INT     4
#define NC_LONG    NC_INT
#define NC_FLOAT   5
#define NC_DOUBLE  6
#define NC_UBYTE   7
#define NC_USHORT  8
#define NC_UINT    9
#define NC_INT64  10
#define NC_UINT64 11
#define NC_STRING 12
#define NC_MAX_ATOMIC_TYPE NC_STRING
#define NC_VLEN     13
#define NC_OPAQUE   14
#define NC_ENUM     15
#define NC_COMPOUND 16
#define NC_FIRSTUSERTYPEID 32

/* default fill values (pnetcdf.h.in:104-116) */
#define NC_FILL_BYTE    ((signed char)-127)
#define NC_FILL_CHAR    ((char)0)
#define NC_FILL_SHORT   ((short)-32767)
#define NC_FILL_INT     (-2147483647)
#define NC_FILL_FLOAT   (9.9692099683868690e+36f)
#define NC_FILL_DOUBLE  (9.9692099683868690e+36)
#define NC_FILL_UBYTE   (255)
#define NC_FILL_USHORT  (65535)
#define NC_FILL_UINT    (4294967295U)
#define NC_FILL_INT64   ((long long)-9223372036854775806LL)
#define NC_FILL_UINT64  ((unsigned long long)18446744073709551614ULL)
#define NC_FILL_STRING  ((char *)"")

/* external type ranges (pnetcdf.h.in:127-146) */
#define NC_MAX_BYTE 127
#define NC_MIN_BYTE (-NC_MAX_BYTE-1)
#define NC_MAX_CHAR 255
#define NC_MAX_SHORT 32767
#define NC_MIN_SHORT (-NC_MAX_SHORT - 1)
#define NC_MAX_INT 2147483647
#define NC_MIN_INT (-NC_MAX_INT - 1)
#define NC_MAX_FLOAT 3.402823466e+38f
#define NC_MIN_FLOAT (-NC_MAX_FLOAT)
#define NC_MAX_DOUBLE 1.7976931348623157e+308
#define NC_MIN_DOUBLE (-NC_MAX_DOUBLE)
#define NC_MAX_UBYTE NC_MAX_CHAR
#define NC_MAX_USHORT 65535U
#define NC_MAX_UINT 4294967295U
#define NC_MAX_INT64 (9223372036854775807LL)
#define NC_MIN_INT64 (-9223372036854775807LL-1LL)
#define NC_MAX_UINT64 (18446744073709551615ULL)

#define NC_FillValue "_FillValue"
#define NC_FILL           0
#define NC_NOFILL         0x100

/* create / open modes (pnetcdf.h.in:168-230) */
#define NC_NOWRITE        0x0000
#define NC_WRITE          0x0001
#define NC_CLOBBER        0x0000
#define NC_NOCLOBBER      0x0004
#define NC_DISKLESS       0x0008
#define NC_MMAP           0x0010
#define NC_64BIT_DATA     0x0020
#define NC_CDF5           NC_64BIT_DATA
#define NC_UDF0           0x0040
#define NC_UDF1           0x0080
#define NC_CLASSIC_MODEL  0x0100
#define NC_64BIT_OFFSET   0x0200
#define NC_LOCK           0x0400
#define NC_SHARE          0x0800
#define NC_NETCDF4        0x1000
#define NC_MPIIO          0x2000
#define NC_MPIPOSIX       NC_MPIIO
#define NC_PNETCDF        (NC_MPIIO)
#define NC_PERSIST        0x4000
#define NC_INMEMORY       0x8000
#define NC_NOATTCREORD    0x20000

/* formats (pnetcdf.h.in:235-290) */
#define NC_FORMAT_CLASSIC      1
#define NC_FORMAT_64BIT_OFFSET 2
#define NC_FORMAT_64BIT           (NC_FORMAT_64BIT_OFFSET)
#define NC_FORMAT_NETCDF4 3
#define NC_FORMAT_NETCDF4_CLASSIC 4
#define NC_FORMAT_64BIT_DATA   5
#define NC_FORMATX_NC3       (1)
#define NC_FORMATX_NC_HDF5   (2)
#define NC_FORMATX_NC4       NC_FORMATX_NC_HDF5
#define NC_FORMATX_PNETCDF   (4)
#define NC_FORMATX_UNDEFINED (0)

#define NC_SIZEHINT_DEFAULT 0
#define NC_ALIGN_CHUNK ((size_t)(-1))
#define NC_UNLIMITED      0L
#define NC_GLOBAL         (-1)
#define NC_MAX_DIMS     NC_MAX_INT
#define NC_MAX_ATTRS    NC_MAX_INT
#define NC_MAX_VARS     NC_MAX_INT
#define NC_MAX_NAME       256
#define NC_MAX_VAR_DIMS NC_MAX_INT

/* errors (pnetcdf.h.in:400-515) */
#define NC_ISSYSERR(err) ((err) > 0)
#define NC_NOERR      0
#define NC2_ERR       (-1)
#define NC_EBADID         (-33)
#define NC_ENFILE         (-34)
#define NC_EEXIST         (-35)
#define NC_EINVAL   (-36)
#define NC_EPERM          (-37)
#define NC_ENOTINDEFINE   (-38)
#define NC_EINDEFINE      (-39)
#define NC_EINVALCOORDS   (-40)
#define NC_EMAXDIMS       (-41)
#define NC_ENAMEINUSE     (-42)
#define NC_ENOTATT        (-43)
#define NC_EMAXATTS       (-44)
#define NC_EBADTYPE (-45)
#define NC_EBADDIM        (-46)
#define NC_EUNLIMPOS      (-47)
#define NC_EMAXVARS       (-48)
#define NC_ENOTVAR        (-49)
#define NC_EGLOBAL        (-50)
#define NC_ENOTNC         (-51)
#define NC_ESTS           (-52)
#define NC_EMAXNAME       (-53)
#define NC_EUNLIMIT       (-54)
#define NC_ENORECVARS     (-55)
#define NC_ECHAR    (-56)
#define NC_EEDGE          (-57)
#define NC_ESTRIDE        (-58)
#define NC_EBADNAME       (-59)
#define NC_ERANGE   (-60)
#define NC_ENOMEM   (-61)
#define NC_EVARSIZE       (-62)
#define NC_EDIMSIZE       (-63)
#define NC_ETRUNC         (-64)
#define NC_EAXISTYPE      (-65)
#define NC_EIO            (-68)
#define NC_ENOTFOUND      (-90)
#define NC_ECANTREMOVE    (-91)
#define NC_EINTERNAL      (-92)
#define NC_EPNETCDF       (-93)
#define NC_ENOTNC3        (-113)
#define NC_ENOPAR         (-114)
#define NC_ENOTBUILT      (-128)
#define NC_EMPI           (-131)
#define NC_ENULLPAD       (-134)
#endif /* _NETCDF_ */

/* PnetCDF-only constants (pnetcdf.h.in:520-600) */
#define NC_REQ_NULL       (-1)
#define NC_COUNT_IGNORE (-1)
#define NC_REQ_ALL        (-1)
#define NC_GET_REQ_ALL    (-2)
#define NC_PUT_REQ_ALL    (-3)
#define NC_MAX_NFILES     1024
#define NC_FORMAT_UNKNOWN (-1)
#define NC_32BIT          0x1000000
#define NC_FORMAT_CDF2    2
#define NC_FORMAT_CDF5    5
#define NC_BP             0x10000
#define NC_FORMAT_BP      6

/* PnetCDF error codes (pnetcdf.h.in:606-690) */
#define NC_ESMALL         (-201)
#define NC_ENOTINDEP      (-202)
#define NC_EINDEP         (-203)
#define NC_EFILE          (-204)
#define NC_EREAD          (-205)
#define NC_EWRITE         (-206)
#define NC_EOFILE         (-207)
#define NC_EMULTITYPES  (-208)   /* pnetcdf.h.in:629 */
#define NC_EIOMISMATCH  (-209)   /* pnetcdf.h.in:630 */
#define NC_ENEGATIVECNT   (-210)
#define NC_EUNSPTETYPE    (-211)
#define NC_EINVAL_REQUEST (-212)
#define NC_EAINT_TOO_SMALL (-213)
#define NC_ENOTSUPPORT    (-214)
#define NC_ENULLBUF       (-215)
#define NC_EPREVATTACHBUF (-216)
#define NC_ENULLABUF      (-217)
#define NC_EPENDINGBPUT   (-218)
#define NC_EINSUFFBUF     (-219)
#define NC_ENOENT         (-220)
#define NC_EINTOVERFLOW   (-221)
#define NC_ENOTENABLED    (-222)
#define NC_EBAD_FILE      (-223)
#define NC_ENO_SPACE      (-224)
#define NC_EQUOTA         (-225)
#define NC_ENULLSTART     (-226)
#define NC_ENULLCOUNT     (-227)
#define NC_EINVAL_CMODE   (-228)
#define NC_ETYPESIZE      (-229)
#define NC_ETYPE_MISMATCH (-230)
#define NC_ETYPESIZE_MISMATCH (-231)
#define NC_ESTRICTCDF2    (-232)
#define NC_ENOTRECVAR     (-233)
#define NC_ENOTFILL       (-234)
#define NC_EINVAL_OMODE   (-235)
#define NC_EPENDING       (-236)
#define NC_EMAX_REQ       (-237)
#define NC_EBADLOG        (-238)
#define NC_EFLUSHED       (-239)
#define NC_EADIOS         (-240)
#define NC_EFSTYPE        (-241)
#define NC_EDRIVER        (-242)
#define NC_EFILEVIEW      (-243)
#define NC_EMULTIDEFINE             (-250)
#define NC_EMULTIDEFINE_OMODE       (-251)
#define NC_EMULTIDEFINE_DIM_NUM     (-252)
#define NC_EMULTIDEFINE_DIM_SIZE    (-253)
#define NC_EMULTIDEFINE_DIM_NAME    (-254)
#define NC_EMULTIDEFINE_VAR_NUM     (-255)
#define NC_EMULTIDEFINE_VAR_NAME    (-256)
#define NC_EMULTIDEFINE_VAR_NDIMS   (-257)
#define NC_EMULTIDEFINE_VAR_DIMIDS  (-258)
#define NC_EMULTIDEFINE_VAR_TYPE    (-259)
#define NC_EMULTIDEFINE_VAR_LEN     (-260)
#define NC_EMULTIDEFINE_NUMRECS     (-261)
#define NC_EMULTIDEFINE_VAR_BEGIN   (-262)
#define NC_EMULTIDEFINE_ATTR_NUM    (-263)
#define NC_EMULTIDEFINE_ATTR_SIZE   (-264)
#define NC_EMULTIDEFINE_ATTR_NAME   (-265)
#define NC_EMULTIDEFINE_ATTR_TYPE   (-266)
#define NC_EMULTIDEFINE_ATTR_LEN    (-267)
#define NC_EMULTIDEFINE_ATTR_VAL    (-268)
#define NC_EMULTIDEFINE_FNC_ARGS    (-269)
#define NC_EMULTIDEFINE_FILL_MODE   (-270)
#define NC_EMULTIDEFINE_VAR_FILL_MODE  (-271)
#define NC_EMULTIDEFINE_VAR_FILL_VALUE (-272)
#define NC_EMULTIDEFINE_CMODE       (-273)
#define NC_EMULTIDEFINE_HINTS       (-274)
#define NC_EMULTIDEFINE_FIRST NC_EMULTIDEFINE
#define NC_EMULTIDEFINE_LAST  NC_EMULTIDEFINE_HINTS
'''

MISC = r'''
const char *ncmpi_strerror(int err);
const char *ncmpi_strerrno(int err);
const char *ncmpi_inq_libvers(void);

/* files (pnetcdf.h.in:740-860) */
int ncmpi_create(MPI_Comm comm, const char *path, int cmode, MPI_Info info, int *ncidp);
int ncmpi_open(MPI_Comm comm, const char *path, int omode, MPI_Info info, int *ncidp);
int ncmpi_inq_file_info(int ncid, MPI_Info *info_used);
int ncmpi_get_file_info(int ncid, MPI_Info *info_used);
int ncmpi_delete(const char *filename, MPI_Info info);
int ncmpi_enddef(int ncid);
int ncmpi__enddef(int ncid, MPI_Offset h_minfree, MPI_Offset v_align, MPI_Offset v_minfree,
                  MPI_Offset r_align);
int ncmpi_redef(int ncid);
int ncmpi_set_default_format(int format, int *old_formatp);
int ncmpi_inq_default_format(int *formatp);
int ncmpi_sync(int ncid);
int ncmpi_flush(int ncid);
int ncmpi_sync_numrecs(int ncid);
int ncmpi_abort(int ncid);
int ncmpi_begin_indep_data(int ncid);
int ncmpi_end_indep_data(int ncid);
int ncmpi_close(int ncid);
int ncmpi_set_fill(int ncid, int fillmode, int *old_modep);
int ncmpi_def_var_fill(int ncid, int varid, int no_fill, const void *fill_value);
int ncmpi_fill_var_rec(int ncid, int varid, MPI_Offset recno);

/* define mode */
int ncmpi_def_dim(int ncid, const char *name, MPI_Offset len, int *idp);
int ncmpi_def_var(int ncid, const char *name, nc_type xtype, int ndims, const int *dimidsp, int *varidp);
int ncmpi_rename_dim(int ncid, int dimid, const char *name);
int ncmpi_rename_var(int ncid, int varid, const char *name);

/* inquiry */
int ncmpi_inq(int ncid, int *ndimsp, int *nvarsp, int *ngattsp, int *unlimdimidp);
int ncmpi_inq_format(int ncid, int *formatp);
int ncmpi_inq_file_format(const char *filename, int *formatp);
int ncmpi_inq_version(int ncid, int *NC_mode);
int ncmpi_inq_striping(int ncid, int *striping_size, int *striping_count);
int ncmpi_inq_ndims(int ncid, int *ndimsp);
int ncmpi_inq_nvars(int ncid, int *nvarsp);
int ncmpi_inq_num_rec_vars(int ncid, int *nvarsp);
int ncmpi_inq_num_fix_vars(int ncid, int *nvarsp);
int ncmpi_inq_natts(int ncid, int *ngattsp);
int ncmpi_inq_unlimdim(int ncid, int *unlimdimidp);
int ncmpi_inq_dimid(int ncid, const char *name, int *idp);
int ncmpi_inq_dim(int ncid, int dimid, char *name, MPI_Offset *lenp);
int ncmpi_inq_dimname(int ncid, int dimid, char *name);
int ncmpi_inq_dimlen(int ncid, int dimid, MPI_Offset *lenp);
int ncmpi_inq_var(int ncid, int varid, char *name, nc_type *xtypep, int *ndimsp, int *dimidsp,
                  int *nattsp);
int ncmpi_inq_varid(int ncid, const char *name, int *varidp);
int ncmpi_inq_varname(int ncid, int varid, char *name);
int ncmpi_inq_vartype(int ncid, int varid, nc_type *xtypep);
int ncmpi_inq_varndims(int ncid, int varid, int *ndimsp);
int ncmpi_inq_vardimid(int ncid, int varid, int *dimidsp);
int ncmpi_inq_varnatts(int ncid, int varid, int *nattsp);
int ncmpi_inq_varoffset(int ncid, int varid, MPI_Offset *offset);
int ncmpi_inq_put_size(int ncid, MPI_Offset *size);
int ncmpi_inq_get_size(int ncid, MPI_Offset *size);
int ncmpi_inq_header_size(int ncid, MPI_Offset *size);
int ncmpi_inq_header_extent(int ncid, MPI_Offset *extent);
int ncmpi_inq_malloc_size(MPI_Offset *size);
int ncmpi_inq_malloc_max_size(MPI_Offset *size);
int ncmpi_inq_malloc_list(void);
int ncmpi_inq_files_opened(int *num, int *ncids);
int ncmpi_inq_recsize(int ncid, MPI_Offset *recsize);
int ncmpi_inq_var_fill(int ncid, int varid, int *no_fill, void *fill_value);
int ncmpi_inq_path(int ncid, int *pathlen, char *path);

/* attributes */
int ncmpi_inq_att(int ncid, int varid, const char *name, nc_type *xtypep, MPI_Offset *lenp);
int ncmpi_inq_attid(int ncid, int varid, const char *name, int *idp);
int ncmpi_inq_atttype(int ncid, int varid, const char *name, nc_type *xtypep);
int ncmpi_inq_attlen(int ncid, int varid, const char *name, MPI_Offset *lenp);
int ncmpi_inq_attname(int ncid, int varid, int attnum, char *name);
int ncmpi_copy_att(int ncid_in, int varid_in, const char *name, int ncid_out, int varid_out);
int ncmpi_rename_att(int ncid, int varid, const char *name, const char *newname);
int ncmpi_del_att(int ncid, int varid, const char *name);
int ncmpi_put_att(int ncid, int varid, const char *name, nc_type xtype, MPI_Offset nelems,
                  const void *value);
int ncmpi_get_att(int ncid, int varid, const char *name, void *value);
int ncmpi_put_att_text(int ncid, int varid, const char *name, MPI_Offset len, const char *op);
int ncmpi_get_att_text(int ncid, int varid, const char *name, char *ip);
int ncmpi_put_att_ubyte(int ncid, int varid, const char *name, nc_type xtype, MPI_Offset len,
                        const unsigned char *op);
int ncmpi_get_att_ubyte(int ncid, int varid, const char *name, unsigned char *ip);

/* nonblocking control (pnetcdf.h.in:2348-2367) */
int ncmpi_wait(int ncid, int count, int array_of_requests[], int array_of_statuses[]);
int ncmpi_wait_all(int ncid, int count, int array_of_requests[], int array_of_statuses[]);
int ncmpi_cancel(int ncid, int num, int *reqs, int *statuses);
int ncmpi_buffer_attach(int ncid, MPI_Offset bufsize);
int ncmpi_buffer_detach(int ncid);
int ncmpi_inq_buffer_usage(int ncid, MPI_Offset *usage);
int ncmpi_inq_buffer_size(int ncid, MPI_Offset *buf_size);
int ncmpi_inq_nreqs(int ncid, int *nreqs);

/* vard: the file layout is an MPI filetype (pnetcdf.h.in:2326-2340) */
int ncmpi_get_vard(int ncid, int varid, MPI_Datatype filetype, void *ip, MPI_Offset bufcount,
                   MPI_Datatype buftype);
int ncmpi_get_vard_all(int ncid, int varid, MPI_Datatype filetype, void *ip, MPI_Offset bufcount,
                       MPI_Datatype buftype);
int ncmpi_put_vard(int ncid, int varid, MPI_Datatype filetype, const void *ip, MPI_Offset bufcount,
                   MPI_Datatype buftype);
int ncmpi_put_vard_all(int ncid, int varid, MPI_Datatype filetype, const void *ip, MPI_Offset bufcount,
                       MPI_Datatype buftype);
'''


def proto(name, args):
    return f"int {name}(int ncid{args});"


def gen():
    out = []
    w = out.append
    w("/*")
    w(" * pnetcdf.h -- the PnetCDF public C API (version 1.15.0) over the MI355X")
    w(" * conversion path.  GENERATED by tools/gen_pnetcdf_h.py; do not edit.")
    w(" *")
    w(" * Every entry point has the reference's name, signature and error codes")
    w(" * (src/include/pnetcdf.h.in).  libpnetcdf.so implements them with a")
    w(" * dispatcher (pnetcdf_amd/csrc/pnc_dispatch.c, restating")
    w(" * src/dispatchers/) over the driver table of include/pncx_dispatch.h")
    w(" * (struct PNC_driver, src/include/dispatch.h:63-125), whose MI355X driver")
    w(" * converts every buffer with the HIP kernels of libpncx.so.")
    w(" */")
    w("#ifndef H_PNETCDF")
    w("#define H_PNETCDF")
    w("")
    w("#include <mpi.h>")
    w(CONSTANTS)
    w("#if defined(__cplusplus)")
    w('extern "C" {')
    w("#endif")
    w(MISC)
    # typed attributes
    w("/* typed attributes (pnetcdf.h.in:960-1060) */")
    for t, c in TYPES[1:]:
        w(f"int ncmpi_put_att_{t}(int ncid, int varid, const char *name, nc_type xtype, MPI_Offset len, "
          f"const {c} *op);")
        w(f"int ncmpi_get_att_{t}(int ncid, int varid, const char *name, {c} *ip);")
    # blocking
    w("")
    w("/* blocking: ncmpi_{put,get}_var{,1,a,s,m}[_<type>][_all] */")
    for kind in ("", "1", "a", "s", "m"):
        for coll in ("", "_all"):
            w(proto(f"ncmpi_put_var{kind}{coll}", f", int varid{KIND_ARGS[kind]}, const void *op, "
                    "MPI_Offset bufcount, MPI_Datatype buftype"))
            w(proto(f"ncmpi_get_var{kind}{coll}", f", int varid{KIND_ARGS[kind]}, void *ip, "
                    "MPI_Offset bufcount, MPI_Datatype buftype"))
        for t, c in TYPES:
            for coll in ("", "_all"):
                w(proto(f"ncmpi_put_var{kind}_{t}{coll}", f", int varid{KIND_ARGS[kind]}, const {c} *op"))
                w(proto(f"ncmpi_get_var{kind}_{t}{coll}", f", int varid{KIND_ARGS[kind]}, {c} *ip"))
    # varn
    w("")
    w("/* varn: num subarrays of one variable */")
    for coll in ("", "_all"):
        w(proto(f"ncmpi_put_varn{coll}", f", int varid{VARN_ARGS}, const void *op, MPI_Offset bufcount, "
                "MPI_Datatype buftype"))
        w(proto(f"ncmpi_get_varn{coll}", f", int varid{VARN_ARGS}, void *ip, MPI_Offset bufcount, "
                "MPI_Datatype buftype"))
    for t, c in TYPES:
        for coll in ("", "_all"):
            w(proto(f"ncmpi_put_varn_{t}{coll}", f", int varid{VARN_ARGS}, const {c} *op"))
            w(proto(f"ncmpi_get_varn_{t}{coll}", f", int varid{VARN_ARGS}, {c} *ip"))
    # nonblocking
    w("")
    w("/* nonblocking: ncmpi_{iput,iget,bput}_var{,1,a,s,m,n}[_<type>] */")
    for kind in ("", "1", "a", "s", "m", "n"):
        ka = VARN_ARGS if kind == "n" else KIND_ARGS[kind]
        w(proto(f"ncmpi_iput_var{kind}", f", int varid{ka}, const void *op, MPI_Offset bufcount, "
                "MPI_Datatype buftype, int *req"))
        w(proto(f"ncmpi_iget_var{kind}", f", int varid{ka}, void *ip, MPI_Offset bufcount, "
                "MPI_Datatype buftype, int *req"))
        w(proto(f"ncmpi_bput_var{kind}", f", int varid{ka}, const void *op, MPI_Offset bufcount, "
                "MPI_Datatype buftype, int *req"))
        for t, c in TYPES:
            w(proto(f"ncmpi_iput_var{kind}_{t}", f", int varid{ka}, const {c} *op, int *req"))
            w(proto(f"ncmpi_iget_var{kind}_{t}", f", int varid{ka}, {c} *ip, int *req"))
            w(proto(f"ncmpi_bput_var{kind}_{t}", f", int varid{ka}, const {c} *op, int *req"))
    # multi-variable
    w("")
    w("/* multi-variable: ncmpi_{mput,mget}_var{,1,a,s,m}[_<type>][_all] */")
    for kind in ("", "1", "a", "s", "m"):
        for coll in ("", "_all"):
            w(proto(f"ncmpi_mput_var{kind}{coll}", f", int num, int *varids{MKIND_ARGS[kind]}, void* const *buf, "
                    "const MPI_Offset *bufcounts, const MPI_Datatype datatypes[]"))
            w(proto(f"ncmpi_mget_var{kind}{coll}", f", int num, int *varids{MKIND_ARGS[kind]}, void *bufs[], "
                    "const MPI_Offset *bufcounts, const MPI_Datatype *datatypes"))
        for t, c in TYPES:
            for coll in ("", "_all"):
                w(proto(f"ncmpi_mput_var{kind}_{t}{coll}", f", int num, int *varids{MKIND_ARGS[kind]}, "
                        f"{c}* const *buf"))
                w(proto(f"ncmpi_mget_var{kind}_{t}{coll}", f", int num, int *varids{MKIND_ARGS[kind]}, "
                        f"{c} *bufs[]"))
    w("")
    w("#if defined(__cplusplus)")
    w("}")
    w("#endif")
    w("#endif /* H_PNETCDF */")
    return "\n".join(out) + "\n"


def main():
    path = os.path.join(ROOT, "include", "pnetcdf.h")
    open(path, "w").write(gen())
    print(path)


if __name__ == "__main__":
    main()
