"""Python mirror of the file-level C-ABI (include/pncx_nc.h).

Functions keep the ncmpi_* names and argument meaning (src/include/pnetcdf.h.in)
and return the NC status code first, as the reference's C tests check it
(EXP_ERR / CHECK_ERR).  Data calls take numpy arrays (host) or torch tensors
(device, *_dev); the in-memory type of the array selects the itype.
"""
import ctypes

import numpy as np

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import pncx

# modes / formats / special ids (pnetcdf.h.in:151-230, 578-615)
NC_NOWRITE, NC_WRITE, NC_CLOBBER, NC_NOCLOBBER = 0x0000, 0x0001, 0x0000, 0x0004
NC_64BIT_DATA, NC_CLASSIC_MODEL, NC_64BIT_OFFSET, NC_NETCDF4 = 0x0020, 0x0100, 0x0200, 0x1000
NC_FILL, NC_NOFILL = 0, 0x100
NC_UNLIMITED, NC_GLOBAL = 0, -1
NC_REQ_NULL, NC_REQ_ALL, NC_GET_REQ_ALL, NC_PUT_REQ_ALL = -1, -1, -2, -3
NC_FORMAT_UNKNOWN, NC_FORMAT_CLASSIC, NC_FORMAT_CDF2 = -1, 1, 2
NC_FORMAT_NETCDF4, NC_FORMAT_NETCDF4_CLASSIC, NC_FORMAT_CDF5 = 3, 4, 5

# errors (pnetcdf.h.in:400-640)
ERR = dict(
    NC_NOERR=0, NC_EBADID=-33, NC_EEXIST=-35, NC_EINVAL=-36, NC_EPERM=-37, NC_ENOTINDEFINE=-38,
    NC_EINDEFINE=-39, NC_EINVALCOORDS=-40, NC_EMAXDIMS=-41, NC_ENAMEINUSE=-42, NC_ENOTATT=-43,
    NC_EMAXATTS=-44, NC_EBADTYPE=-45, NC_EBADDIM=-46, NC_EUNLIMPOS=-47, NC_EMAXVARS=-48,
    NC_ENOTVAR=-49, NC_EGLOBAL=-50, NC_ENOTNC=-51, NC_EMAXNAME=-53, NC_EUNLIMIT=-54, NC_ECHAR=-56,
    NC_EEDGE=-57, NC_ESTRIDE=-58, NC_EBADNAME=-59, NC_ERANGE=-60, NC_ENOMEM=-61, NC_EVARSIZE=-62,
    NC_EDIMSIZE=-63, NC_ENOTNC3=-113, NC_ENOTBUILT=-128, NC_ENULLPAD=-134, NC_EFILE=-204,
    NC_EREAD=-205, NC_EWRITE=-206, NC_EMULTITYPES=-208, NC_EIOMISMATCH=-209, NC_ENEGATIVECNT=-210, NC_EINVAL_REQUEST=-212, NC_EPREVATTACHBUF=-216,
    NC_ENULLABUF=-217, NC_EPENDINGBPUT=-218, NC_EINSUFFBUF=-219, NC_ENOENT=-220,
    NC_EINTOVERFLOW=-221, NC_ENULLSTART=-226, NC_EINVAL_CMODE=-228, NC_ESTRICTCDF2=-232, NC_ENOTRECVAR=-233,
    NC_ENOTFILL=-234, NC_EINVAL_OMODE=-235, NC_EPENDING=-236, PNCX_EDEVICE=-1900)
globals().update(ERR)
ERRNAME = {v: k for k, v in ERR.items()}

_DTYPE_ITYPE = {
    np.dtype(np.int8): T.ITYPE_SCHAR, np.dtype(np.uint8): T.ITYPE_UCHAR,
    np.dtype(np.int16): T.ITYPE_SHORT, np.dtype(np.uint16): T.ITYPE_USHORT,
    np.dtype(np.int32): T.ITYPE_INT, np.dtype(np.uint32): T.ITYPE_UINT,
    np.dtype(np.int64): T.ITYPE_LONGLONG, np.dtype(np.uint64): T.ITYPE_ULONGLONG,
    np.dtype(np.float32): T.ITYPE_FLOAT, np.dtype(np.float64): T.ITYPE_DOUBLE,
    np.dtype("S1"): T.ITYPE_CHAR,
}
_TORCH_ITYPE = None

_sig_done = False


def lib():
    global _sig_done
    L = pncx.lib()
    if _sig_done:
        return L
    vp, ll, i, cp = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_char_p
    ip = ctypes.POINTER(ctypes.c_int)
    lp = ctypes.POINTER(ctypes.c_longlong)
    sig = {
        "pncx_nc_inq_file_format": [cp, ip], "pncx_nc_create": [cp, i, ip], "pncx_nc_open": [cp, i, ip],
        "pncx_nc_validate": [cp], "pncx_nc_redef": [i], "pncx_nc_enddef": [i],
        "pncx_nc__enddef": [i, ll, ll, ll, ll], "pncx_nc_sync": [i], "pncx_nc_close": [i],
        "pncx_nc_sync_numrecs": [i, ll],
        "pncx_nc_def_dim": [i, cp, ll, ip], "pncx_nc_def_var": [i, cp, i, i, ip, ip],
        "pncx_nc_rename_dim": [i, i, cp], "pncx_nc_rename_var": [i, i, cp],
        "pncx_nc_set_fill": [i, i, ip], "pncx_nc_def_var_fill": [i, i, i, vp],
        "pncx_nc_inq_var_fill": [i, i, ip, vp], "pncx_nc_fill_var_rec": [i, i, ll],
        "pncx_nc_put_att": [i, i, cp, i, ll, vp, i], "pncx_nc_get_att": [i, i, cp, vp, i],
        "pncx_nc_del_att": [i, i, cp], "pncx_nc_rename_att": [i, i, cp, cp],
        "pncx_nc_inq": [i, ip, ip, ip, ip], "pncx_nc_inq_format": [i, ip],
        "pncx_nc_inq_dim": [i, i, cp, lp], "pncx_nc_inq_dimid": [i, cp, ip],
        "pncx_nc_inq_var": [i, i, cp, ip, ip, ip, ip], "pncx_nc_inq_varid": [i, cp, ip],
        "pncx_nc_inq_varoffset": [i, i, lp], "pncx_nc_inq_att": [i, i, cp, ip, lp],
        "pncx_nc_inq_attname": [i, i, i, cp], "pncx_nc_inq_header_size": [i, lp],
        "pncx_nc_inq_header_extent": [i, lp], "pncx_nc_inq_recsize": [i, lp],
        "pncx_nc_inq_io_size": [i, lp, lp],
        "pncx_nc_put_varm": [i, i, vp, vp, vp, vp, vp, i], "pncx_nc_get_varm": [i, i, vp, vp, vp, vp, vp, i],
        "pncx_nc_put_varm_dev": [i, i, vp, vp, vp, vp, vp, i, vp],
        "pncx_nc_get_varm_dev": [i, i, vp, vp, vp, vp, vp, i, vp],
        "pncx_nc_iput_varm": [i, i, vp, vp, vp, vp, vp, i, ip],
        "pncx_nc_iget_varm": [i, i, vp, vp, vp, vp, vp, i, ip],
        "pncx_nc_wait_all": [i, i, vp, vp], "pncx_nc_cancel": [i, i, vp, vp], "pncx_nc_inq_nreqs": [i, ip],
        "pncx_nc_buffer_attach": [i, ll], "pncx_nc_buffer_detach": [i],
        "pncx_nc_inq_buffer_size": [i, lp], "pncx_nc_inq_buffer_usage": [i, lp],
        "pncx_nc_bput_varm": [i, i, vp, vp, vp, vp, vp, i, ip],
        "pncx_nc_put_varm_flex": [i, i, vp, vp, vp, vp, vp, ll, vp],
        "pncx_nc_get_varm_flex": [i, i, vp, vp, vp, vp, vp, ll, vp],
        "pncx_nc_put_varm_flex_dev": [i, i, vp, vp, vp, vp, vp, ll, vp, vp],
        "pncx_nc_get_varm_flex_dev": [i, i, vp, vp, vp, vp, vp, ll, vp, vp],
        "pncx_nc_iput_varm_flex": [i, i, vp, vp, vp, vp, vp, ll, vp, ip],
        "pncx_nc_iget_varm_flex": [i, i, vp, vp, vp, vp, vp, ll, vp, ip],
        "pncx_nc_put_varn": [i, i, i, vp, vp, vp, i], "pncx_nc_get_varn": [i, i, i, vp, vp, vp, i],
        "pncx_nc_iput_varn": [i, i, i, vp, vp, vp, i, ip], "pncx_nc_iget_varn": [i, i, i, vp, vp, vp, i, ip],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.restype = ctypes.c_int
        f.argtypes = args
    _sig_done = True
    return L


def strerror(err):
    return ERRNAME.get(err, pncx.strerror(err))


def _b(s):
    # names read from a file are not validated (hdr_get_NC_name does not
    # check them either); surrogateescape round-trips non-UTF-8 bytes
    return s.encode("utf-8", "surrogateescape") if isinstance(s, str) else s


def _offs(vals):
    """int64 array + pointer (None -> NULL); the array must be kept alive"""
    if vals is None:
        return None, None
    a = np.ascontiguousarray(np.asarray(vals, dtype=np.int64).reshape(-1))
    return a, ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(a.ctypes.data)


def itype_of(arr):
    dt = np.dtype(arr.dtype)
    if dt.kind == "S":
        return T.ITYPE_CHAR
    return _DTYPE_ITYPE[dt]


def torch_itype(t):
    import torch
    m = {torch.int8: T.ITYPE_SCHAR, torch.uint8: T.ITYPE_UCHAR, torch.int16: T.ITYPE_SHORT,
         torch.int32: T.ITYPE_INT, torch.int64: T.ITYPE_LONGLONG, torch.float32: T.ITYPE_FLOAT,
         torch.float64: T.ITYPE_DOUBLE}
    for name, it in (("uint16", T.ITYPE_USHORT), ("uint32", T.ITYPE_UINT), ("uint64", T.ITYPE_ULONGLONG)):
        if hasattr(torch, name):
            m[getattr(torch, name)] = it
    return m[t.dtype]


# ------------------------------------------------------------------ files
def inq_file_format(path):
    f = ctypes.c_int()
    err = lib().pncx_nc_inq_file_format(_b(path), ctypes.byref(f))
    return err, f.value


def create(path, cmode=0):
    n = ctypes.c_int(-1)
    err = lib().pncx_nc_create(_b(path), cmode, ctypes.byref(n))
    return err, n.value


def open(path, omode=0):  # noqa: A001  (mirrors ncmpi_open)
    n = ctypes.c_int(-1)
    err = lib().pncx_nc_open(_b(path), omode, ctypes.byref(n))
    return err, n.value


def validate(path):
    return lib().pncx_nc_validate(_b(path))


def redef(ncid):
    return lib().pncx_nc_redef(ncid)


def enddef(ncid):
    return lib().pncx_nc_enddef(ncid)


def _enddef(ncid, h_minfree=0, v_align=0, v_minfree=0, r_align=0):
    return lib().pncx_nc__enddef(ncid, h_minfree, v_align, v_minfree, r_align)


def sync(ncid):
    return lib().pncx_nc_sync(ncid)


def sync_numrecs(ncid, numrecs):
    return lib().pncx_nc_sync_numrecs(ncid, numrecs)


def close(ncid):
    return lib().pncx_nc_close(ncid)


# ------------------------------------------------------------------ define mode
def def_dim(ncid, name, length):
    d = ctypes.c_int(-1)
    err = lib().pncx_nc_def_dim(ncid, _b(name), length, ctypes.byref(d))
    return err, d.value


def def_var(ncid, name, xtype, dimids):
    ids = (ctypes.c_int * max(1, len(dimids)))(*dimids)
    v = ctypes.c_int(-1)
    err = lib().pncx_nc_def_var(ncid, _b(name), xtype, len(dimids), ids if dimids else None, ctypes.byref(v))
    return err, v.value


def rename_dim(ncid, dimid, name):
    return lib().pncx_nc_rename_dim(ncid, dimid, _b(name))


def rename_var(ncid, varid, name):
    return lib().pncx_nc_rename_var(ncid, varid, _b(name))


def set_fill(ncid, mode):
    old = ctypes.c_int()
    err = lib().pncx_nc_set_fill(ncid, mode, ctypes.byref(old))
    return err, old.value


def def_var_fill(ncid, varid, no_fill, fill_value=None):
    """fill_value: a numpy scalar/1-element array of the variable's type (native order)"""
    fv = None if fill_value is None else np.ascontiguousarray(np.asarray(fill_value).reshape(1))
    return lib().pncx_nc_def_var_fill(ncid, varid, int(no_fill), None if fv is None else fv.ctypes.data)


def inq_var_fill(ncid, varid, dtype):
    nf = ctypes.c_int()
    fv = np.zeros(1, dtype=dtype)
    err = lib().pncx_nc_inq_var_fill(ncid, varid, ctypes.byref(nf), fv.ctypes.data)
    return err, nf.value, fv[0]


def fill_var_rec(ncid, varid, recno):
    return lib().pncx_nc_fill_var_rec(ncid, varid, recno)


# ------------------------------------------------------------------ attributes
def put_att(ncid, varid, name, xtype, values, itype=None):
    if isinstance(values, (str, bytes)):
        b = _b(values)
        arr = np.frombuffer(b, dtype="S1") if b else np.zeros(0, dtype="S1")
    else:
        arr = np.ascontiguousarray(np.asarray(values).reshape(-1))
    it = itype if itype is not None else itype_of(arr)
    ptr = arr.ctypes.data if arr.size else None
    return lib().pncx_nc_put_att(ncid, varid, _b(name), xtype, arr.size, ptr, it)


def put_att_text(ncid, varid, name, text):
    return put_att(ncid, varid, name, T.NC_CHAR, text, T.ITYPE_CHAR)


def inq_att(ncid, varid, name):
    xt, n = ctypes.c_int(), ctypes.c_longlong()
    err = lib().pncx_nc_inq_att(ncid, varid, _b(name), ctypes.byref(xt), ctypes.byref(n))
    return err, xt.value, n.value


def get_att(ncid, varid, name, dtype=None):
    """returns (err, values); text attributes come back as bytes"""
    err, xt, n = inq_att(ncid, varid, name)
    if err:
        return err, None
    if xt == T.NC_CHAR and dtype is None:
        out = np.zeros(max(n, 1), dtype="S1")
        err = lib().pncx_nc_get_att(ncid, varid, _b(name), out.ctypes.data, T.ITYPE_CHAR)
        return err, out[:n].tobytes()
    dt = np.dtype(dtype if dtype is not None else T.XTYPE_NP[xt])
    out = np.zeros(max(n, 1), dtype=dt)
    err = lib().pncx_nc_get_att(ncid, varid, _b(name), out.ctypes.data, _DTYPE_ITYPE[dt])
    return err, out[:n]


def del_att(ncid, varid, name):
    return lib().pncx_nc_del_att(ncid, varid, _b(name))


def rename_att(ncid, varid, name, newname):
    return lib().pncx_nc_rename_att(ncid, varid, _b(name), _b(newname))


# ------------------------------------------------------------------ inquiry
def inq(ncid):
    a = [ctypes.c_int() for _ in range(4)]
    err = lib().pncx_nc_inq(ncid, *[ctypes.byref(x) for x in a])
    return (err,) + tuple(x.value for x in a)


def inq_format(ncid):
    f = ctypes.c_int()
    err = lib().pncx_nc_inq_format(ncid, ctypes.byref(f))
    return err, f.value


def inq_dim(ncid, dimid):
    name = ctypes.create_string_buffer(T_MAX_NAME + 1)
    n = ctypes.c_longlong()
    err = lib().pncx_nc_inq_dim(ncid, dimid, name, ctypes.byref(n))
    return err, name.value.decode("utf-8", "surrogateescape"), n.value


def inq_dimid(ncid, name):
    d = ctypes.c_int(-1)
    err = lib().pncx_nc_inq_dimid(ncid, _b(name), ctypes.byref(d))
    return err, d.value


def inq_var(ncid, varid):
    name = ctypes.create_string_buffer(T_MAX_NAME + 1)
    xt, nd, na = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    err = lib().pncx_nc_inq_var(ncid, varid, name, ctypes.byref(xt), ctypes.byref(nd), None, ctypes.byref(na))
    if err:
        return err, None, None, None, None
    dims = (ctypes.c_int * max(1, nd.value))()
    lib().pncx_nc_inq_var(ncid, varid, None, None, None, dims, None)
    return err, name.value.decode("utf-8", "surrogateescape"), xt.value, list(dims)[:nd.value], na.value


def inq_varid(ncid, name):
    v = ctypes.c_int(-1)
    err = lib().pncx_nc_inq_varid(ncid, _b(name), ctypes.byref(v))
    return err, v.value


def inq_varoffset(ncid, varid):
    o = ctypes.c_longlong()
    err = lib().pncx_nc_inq_varoffset(ncid, varid, ctypes.byref(o))
    return err, o.value


def inq_attname(ncid, varid, attnum):
    name = ctypes.create_string_buffer(T_MAX_NAME + 1)
    err = lib().pncx_nc_inq_attname(ncid, varid, attnum, name)
    return err, name.value.decode("utf-8", "surrogateescape")


def inq_header_size(ncid):
    o = ctypes.c_longlong()
    return lib().pncx_nc_inq_header_size(ncid, ctypes.byref(o)), o.value


def inq_header_extent(ncid):
    o = ctypes.c_longlong()
    return lib().pncx_nc_inq_header_extent(ncid, ctypes.byref(o)), o.value


def inq_recsize(ncid):
    o = ctypes.c_longlong()
    return lib().pncx_nc_inq_recsize(ncid, ctypes.byref(o)), o.value


def inq_io_size(ncid):
    p, g = ctypes.c_longlong(), ctypes.c_longlong()
    err = lib().pncx_nc_inq_io_size(ncid, ctypes.byref(p), ctypes.byref(g))
    return err, p.value, g.value


T_MAX_NAME = 256


# ------------------------------------------------------------------ data
def _args(start, count, stride, imap):
    keep = [_offs(x) for x in (start, count, stride, imap)]
    return keep, [k[1] for k in keep]


def put_var(ncid, varid, buf, start=None, count=None, stride=None, imap=None, itype=None):
    """ncmpi_put_var / var1 / vara / vars / varm (selected by which of
    start/count/stride/imap are given) from a host numpy buffer"""
    buf = np.ascontiguousarray(buf)
    keep, a = _args(start, count, stride, imap)
    it = itype if itype is not None else itype_of(buf)
    return lib().pncx_nc_put_varm(ncid, varid, *a, buf.ctypes.data if buf.size else None, it)


def get_var(ncid, varid, out, start=None, count=None, stride=None, imap=None, itype=None):
    assert out.flags["C_CONTIGUOUS"]
    keep, a = _args(start, count, stride, imap)
    it = itype if itype is not None else itype_of(out)
    return lib().pncx_nc_get_varm(ncid, varid, *a, out.ctypes.data if out.size else None, it)


def put_var_dev(ncid, varid, t, start=None, count=None, stride=None, imap=None, stream=None):
    import torch
    keep, a = _args(start, count, stride, imap)
    s = stream if stream is not None else torch.cuda.current_stream()
    return lib().pncx_nc_put_varm_dev(ncid, varid, *a, t.data_ptr() if t.numel() else None, torch_itype(t),
                                      ctypes.c_void_p(s.cuda_stream))


def get_var_dev(ncid, varid, t, start=None, count=None, stride=None, imap=None, stream=None):
    import torch
    keep, a = _args(start, count, stride, imap)
    s = stream if stream is not None else torch.cuda.current_stream()
    return lib().pncx_nc_get_varm_dev(ncid, varid, *a, t.data_ptr() if t.numel() else None, torch_itype(t),
                                      ctypes.c_void_p(s.cuda_stream))


def _nb_contig(buf):
    """A nonblocking request keeps the raw pointer until wait: a strided view
    would be read or written as if packed, and a contiguous copy would die
    before the wait, so the caller must pass a C-contiguous array."""
    if not buf.flags["C_CONTIGUOUS"]:
        raise ValueError("nonblocking requests need a C-contiguous buffer that lives until wait")


def iput_var(ncid, varid, buf, start=None, count=None, stride=None, imap=None, itype=None):
    """ncmpi_iput_var*: the buffer must stay alive and unchanged until wait"""
    _nb_contig(buf)
    keep, a = _args(start, count, stride, imap)
    it = itype if itype is not None else itype_of(buf)
    r = ctypes.c_int(NC_REQ_NULL)
    err = lib().pncx_nc_iput_varm(ncid, varid, *a, buf.ctypes.data if buf.size else None, it, ctypes.byref(r))
    return err, r.value


def iget_var(ncid, varid, out, start=None, count=None, stride=None, imap=None, itype=None):
    _nb_contig(out)
    keep, a = _args(start, count, stride, imap)
    it = itype if itype is not None else itype_of(out)
    r = ctypes.c_int(NC_REQ_NULL)
    err = lib().pncx_nc_iget_varm(ncid, varid, *a, out.ctypes.data if out.size else None, it, ctypes.byref(r))
    return err, r.value


# flexible API: buf holds `bufcount` copies of `buftype` (a pncx.DType, or
# None for MPI_DATATYPE_NULL) starting `base` bytes into the numpy/torch buffer
def _h(buftype):
    return None if buftype is None else buftype.handle


def put_var_flex(ncid, varid, buf, bufcount, buftype, start=None, count=None, stride=None, imap=None, base=0):
    keep, a = _args(start, count, stride, imap)
    return lib().pncx_nc_put_varm_flex(ncid, varid, *a, buf.ctypes.data + base, bufcount, _h(buftype))


def get_var_flex(ncid, varid, out, bufcount, buftype, start=None, count=None, stride=None, imap=None, base=0):
    keep, a = _args(start, count, stride, imap)
    return lib().pncx_nc_get_varm_flex(ncid, varid, *a, out.ctypes.data + base, bufcount, _h(buftype))


def put_var_flex_dev(ncid, varid, t, bufcount, buftype, start=None, count=None, stride=None, imap=None, base=0,
                     stream=None):
    import torch
    keep, a = _args(start, count, stride, imap)
    s = stream if stream is not None else torch.cuda.current_stream()
    return lib().pncx_nc_put_varm_flex_dev(ncid, varid, *a, t.data_ptr() + base, bufcount, _h(buftype),
                                           ctypes.c_void_p(s.cuda_stream))


def get_var_flex_dev(ncid, varid, t, bufcount, buftype, start=None, count=None, stride=None, imap=None, base=0,
                     stream=None):
    import torch
    keep, a = _args(start, count, stride, imap)
    s = stream if stream is not None else torch.cuda.current_stream()
    return lib().pncx_nc_get_varm_flex_dev(ncid, varid, *a, t.data_ptr() + base, bufcount, _h(buftype),
                                           ctypes.c_void_p(s.cuda_stream))


def iput_var_flex(ncid, varid, buf, bufcount, buftype, start=None, count=None, stride=None, imap=None, base=0):
    keep, a = _args(start, count, stride, imap)
    r = ctypes.c_int(NC_REQ_NULL)
    err = lib().pncx_nc_iput_varm_flex(ncid, varid, *a, buf.ctypes.data + base, bufcount, _h(buftype),
                                       ctypes.byref(r))
    return err, r.value


def iget_var_flex(ncid, varid, out, bufcount, buftype, start=None, count=None, stride=None, imap=None, base=0):
    keep, a = _args(start, count, stride, imap)
    r = ctypes.c_int(NC_REQ_NULL)
    err = lib().pncx_nc_iget_varm_flex(ncid, varid, *a, out.ctypes.data + base, bufcount, _h(buftype),
                                       ctypes.byref(r))
    return err, r.value


def _ptr_array(lists):
    """(keep-alive, pointer) for an array of int64 vectors (starts/counts of varn);
    None entries become NULL"""
    if lists is None:
        return None, None
    arrs = [None if x is None else np.ascontiguousarray(np.asarray(x, dtype=np.int64)) for x in lists]
    ptrs = (ctypes.c_void_p * max(1, len(arrs)))(*[None if a is None else a.ctypes.data for a in arrs])
    return (arrs, ptrs), ctypes.cast(ptrs, ctypes.c_void_p)


def put_varn(ncid, varid, starts, counts, buf, itype=None):
    """ncmpi_put_varn: len(starts) subarrays packed one after another in buf"""
    buf = np.ascontiguousarray(buf)
    ks, ps = _ptr_array(starts)
    kc, pc = _ptr_array(counts)
    it = itype if itype is not None else itype_of(buf)
    return lib().pncx_nc_put_varn(ncid, varid, len(starts) if starts is not None else 0, ps, pc,
                                  buf.ctypes.data if buf.size else None, it)


def get_varn(ncid, varid, starts, counts, out, itype=None):
    assert out.flags["C_CONTIGUOUS"]
    ks, ps = _ptr_array(starts)
    kc, pc = _ptr_array(counts)
    it = itype if itype is not None else itype_of(out)
    return lib().pncx_nc_get_varn(ncid, varid, len(starts) if starts is not None else 0, ps, pc,
                                  out.ctypes.data if out.size else None, it)


def iput_varn(ncid, varid, starts, counts, buf, itype=None):
    _nb_contig(buf)
    ks, ps = _ptr_array(starts)
    kc, pc = _ptr_array(counts)
    it = itype if itype is not None else itype_of(buf)
    r = ctypes.c_int(NC_REQ_NULL)
    err = lib().pncx_nc_iput_varn(ncid, varid, len(starts), ps, pc, buf.ctypes.data if buf.size else None, it,
                                  ctypes.byref(r))
    return err, r.value


def iget_varn(ncid, varid, starts, counts, out, itype=None):
    _nb_contig(out)
    ks, ps = _ptr_array(starts)
    kc, pc = _ptr_array(counts)
    it = itype if itype is not None else itype_of(out)
    r = ctypes.c_int(NC_REQ_NULL)
    err = lib().pncx_nc_iget_varn(ncid, varid, len(starts), ps, pc, out.ctypes.data if out.size else None, it,
                                  ctypes.byref(r))
    return err, r.value


def buffer_attach(ncid, size):
    return lib().pncx_nc_buffer_attach(ncid, size)


def buffer_detach(ncid):
    return lib().pncx_nc_buffer_detach(ncid)


def inq_buffer_size(ncid):
    o = ctypes.c_longlong()
    return lib().pncx_nc_inq_buffer_size(ncid, ctypes.byref(o)), o.value


def inq_buffer_usage(ncid):
    o = ctypes.c_longlong()
    return lib().pncx_nc_inq_buffer_usage(ncid, ctypes.byref(o)), o.value


def bput_var(ncid, varid, buf, start=None, count=None, stride=None, imap=None, itype=None):
    """ncmpi_bput_var*: converted into the attached buffer now; buf is free on return"""
    buf = np.ascontiguousarray(buf)
    keep, a = _args(start, count, stride, imap)
    it = itype if itype is not None else itype_of(buf)
    r = ctypes.c_int(NC_REQ_NULL)
    err = lib().pncx_nc_bput_varm(ncid, varid, *a, buf.ctypes.data if buf.size else None, it, ctypes.byref(r))
    return err, r.value


def wait_all(ncid, reqids=None):
    """reqids None -> NC_REQ_ALL; returns (err, statuses)"""
    if reqids is None:
        return lib().pncx_nc_wait_all(ncid, NC_REQ_ALL, None, None), []
    ids = (ctypes.c_int * max(1, len(reqids)))(*reqids)
    st = (ctypes.c_int * max(1, len(reqids)))()
    err = lib().pncx_nc_wait_all(ncid, len(reqids), ids, st)
    return err, list(st)[:len(reqids)]


def cancel(ncid, reqids=None):
    if reqids is None:
        return lib().pncx_nc_cancel(ncid, NC_REQ_ALL, None, None), []
    ids = (ctypes.c_int * max(1, len(reqids)))(*reqids)
    st = (ctypes.c_int * max(1, len(reqids)))()
    err = lib().pncx_nc_cancel(ncid, len(reqids), ids, st)
    return err, list(st)[:len(reqids)]


def inq_nreqs(ncid):
    n = ctypes.c_int()
    err = lib().pncx_nc_inq_nreqs(ncid, ctypes.byref(n))
    return err, n.value
