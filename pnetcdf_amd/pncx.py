"""Python mirror of PnetCDF's conversion interface over the HIP C-ABI.

Names follow the reference (src/drivers/include/common.h:147-221):
``need_convert``, ``in_swapn``, ``putn``, ``getn`` operate on host (numpy)
buffers exactly like ncmpii_need_convert / ncmpii_in_swapn /
ncmpii_putn_NC_<X> / ncmpii_getn_NC_<X>; the ``dev_*`` variants operate on
HBM-resident torch tensors.  Every call goes to ``pnetcdf_amd/lib/libpncx.so``
(the HIP kernels).  There is no CPU fallback: if the library or a GPU is
missing, calls raise.
"""
import ctypes
import os

import numpy as np

from . import nctypes as T

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")
LIB_PATH = os.environ.get("PNCX_LIB_PATH") or os.path.join(LIB_DIR, "libpncx.so")   # override: tools/asan
_lib = None


class PncxError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})" if what else f"{strerror(code)} ({code})")


def lib():
    """Load the in-tree libpncx.so.  torch is imported first (when present)
    so that the library binds to the same HIP runtime instance as torch."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.environ.get("PNCX_NO_TORCH"):          # set only by the host-only ASan run
        try:
            import torch  # noqa: F401  (share one HIP runtime with torch)
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise PncxError(T.PNCX_EDEVICE, f"{LIB_PATH} not built (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, ll, i = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int
    sig = {
        "pncx_xlen": (i, [i]), "pncx_ilen": (i, [i]),
        "pncx_need_convert": (i, [i, i, i]), "pncx_need_swap": (i, [i, i]),
        "pncx_in_swapn": (i, [vp, ll, i]),
        "pncx_putn": (i, [i, i, vp, vp, ll, i, vp]),
        "pncx_getn": (i, [i, i, vp, vp, ll, i]),
        "pncx_dev_in_swapn": (i, [vp, ll, i, vp]),
        "pncx_dev_swapn": (i, [vp, vp, ll, i, vp]),
        "pncx_dev_putn": (i, [i, i, vp, vp, ll, i, vp, vp, vp]),
        "pncx_dev_getn": (i, [i, i, vp, vp, ll, i, vp, vp]),
        "pncx_dev_batch": (i, [vp, i, vp, vp]),
        "pncx_dev_putn_imap": (i, [i, i, vp, vp, i, vp, vp, i, vp, vp, vp]),
        "pncx_dev_getn_imap": (i, [i, i, vp, vp, i, vp, vp, i, vp, vp]),
        "pncx_putn_imap": (i, [i, i, vp, vp, i, vp, vp, i, vp]),
        "pncx_getn_imap": (i, [i, i, vp, vp, i, vp, vp, i]),
        "pncx_batch": (i, [vp, i, vp]),
        "pncx_type_commit": (i, [i, ll, vp, vp, ll, vp]),
        "pncx_type_free": (i, [vp]),
        "pncx_type_inq": (i, [vp, vp, vp, vp, vp]),
        "pncx_putn_flex": (i, [i, i, vp, vp, i, vp, vp, ll, vp, vp]),
        "pncx_getn_flex": (i, [i, i, vp, vp, i, vp, vp, ll, vp]),
        "pncx_dev_putn_flex": (i, [i, i, vp, vp, i, vp, vp, ll, vp, vp, vp, vp]),
        "pncx_dev_getn_flex": (i, [i, i, vp, vp, i, vp, vp, ll, vp, vp, vp]),
        "pncx_dev_fill": (i, [i, vp, ll, vp, vp]),
        "pncx_fill": (i, [i, vp, ll, vp]),
        "pncx_device_count": (i, []), "pncx_set_device": (i, [i]),
        "pncx_get_device": (i, []),
        "pncx_host_register": (i, [vp, ll]), "pncx_host_unregister": (i, [vp]),
        "pncx_dev_status_read": (i, [vp, vp]),
        "pncx_strerror": (ctypes.c_char_p, [i]),
        "pncx_version": (ctypes.c_char_p, []),
        "pncx_knob_set": (i, [ctypes.c_char_p, ll]),
        "pncx_knob_get": (i, [ctypes.c_char_p, ctypes.POINTER(ll)]),
        "pncx_phases": (i, [i]),
        "pncx_phase_name": (ctypes.c_char_p, [i]),
        "pncx_phase_read": (i, [i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ll)]),
    }
    for name, (res, args) in sig.items():
        try:
            f = getattr(L, name)
        except AttributeError:
            # an older build loaded through PNCX_LIB_PATH for an A/B run may
            # lack the round-4 measurement aids; the product build has all
            if os.environ.get("PNCX_LIB_PATH") and name.startswith(("pncx_knob", "pncx_phase")):
                continue
            raise
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def strerror(code):
    try:
        return lib().pncx_strerror(code).decode()
    except Exception:  # library not loadable
        return f"error {code}"


def version():
    return lib().pncx_version().decode()


def device_count():
    return lib().pncx_device_count()


def knob_set(name, value):
    """Set an A/B knob (pncx_knob_set; name as in PNCX_<name>, -1 = default)."""
    _check(lib().pncx_knob_set(name.encode(), int(value)), f"knob_set {name}", (T.NC_NOERR,))


def knob_get(name):
    v = ctypes.c_longlong(0)
    _check(lib().pncx_knob_get(name.encode(), ctypes.byref(v)), f"knob_get {name}", (T.NC_NOERR,))
    return v.value


def phases(enable):
    """Turn per-phase timing of the host-buffer paths on (clearing it) or off."""
    lib().pncx_phases(1 if enable else 0)


def phase_sums():
    """{phase name: (microseconds, count)} of the phases that ran."""
    L, out, i = lib(), {}, 0
    while True:
        nm = L.pncx_phase_name(i)
        if nm is None:
            return out
        us, n = ctypes.c_double(0), ctypes.c_longlong(0)
        L.pncx_phase_read(i, ctypes.byref(us), ctypes.byref(n))
        if n.value:
            out[nm.decode()] = (us.value, n.value)
        i += 1


class Seg(ctypes.Structure):
    """struct pncx_seg (include/pncx.h)"""
    _fields_ = [("dir", ctypes.c_int), ("cdf_ver", ctypes.c_int), ("xtype", ctypes.c_int),
                ("itype", ctypes.c_int), ("nelems", ctypes.c_longlong),
                ("xbuf", ctypes.c_void_p), ("ibuf", ctypes.c_void_p), ("fillp", ctypes.c_void_p)]


def host_register(buf):
    """Pin a long-lived host numpy buffer for direct DMA (pncx_host_register)."""
    _check(lib().pncx_host_register(_np_ptr(buf), buf.nbytes), "host_register", (T.NC_NOERR,))


def host_unregister(buf):
    _check(lib().pncx_host_unregister(_np_ptr(buf)), "host_unregister", (T.NC_NOERR,))


def _np_ptr(a):
    assert isinstance(a, np.ndarray) and a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def _check(code, what, allow=(T.NC_NOERR, T.NC_ERANGE)):
    if code not in allow:
        raise PncxError(code, what)
    return code


# ---------------------------------------------------------------- host side
def need_convert(fmt, xtype, itype):
    """ncmpii_need_convert (convert_swap.m4:85-116)"""
    return lib().pncx_need_convert(fmt, xtype, itype)


def need_swap(xtype, itype):
    """NEED_BYTE_SWAP (common.h:47-54)"""
    return lib().pncx_need_swap(xtype, itype)


def in_swapn(buf, nelems, esize):
    """ncmpii_in_swapn (convert_swap.m4:137-197) on a host numpy buffer."""
    _check(lib().pncx_in_swapn(_np_ptr(buf), nelems, esize), "in_swapn", (T.NC_NOERR,))


def putn(cdf_ver, xtype, xbuf, ibuf, nelems, itype, fillp=None):
    """ncmpii_putn_NC_<X>: ibuf (itype) -> xbuf (big-endian xtype).
    fillp: bytes of the xtype fill value in native order, or None (NULL).
    Returns NC_NOERR or NC_ERANGE; raises on any other status."""
    fb = None if fillp is None else np.frombuffer(bytes(fillp) + b"\0" * 8, np.uint8).copy()
    return _check(lib().pncx_putn(cdf_ver, xtype, _np_ptr(xbuf), _np_ptr(ibuf), nelems, itype,
                                  None if fb is None else _np_ptr(fb)), "putn")


def getn(cdf_ver, xtype, xbuf, ibuf, nelems, itype):
    """ncmpii_getn_NC_<X>: xbuf (big-endian xtype) -> ibuf (itype)."""
    return _check(lib().pncx_getn(cdf_ver, xtype, _np_ptr(xbuf), _np_ptr(ibuf), nelems, itype),
                  "getn")


def fill(xtype, xbuf, nelems, xvalue=None):
    """fill_var_buf (ncmpio_fill.c:89-140) into a host buffer; xvalue = the
    external (big-endian) bytes of a _FillValue, None for the default."""
    xv = None if xvalue is None else np.frombuffer(bytes(xvalue) + b"\0" * 8, np.uint8).copy()
    _check(lib().pncx_fill(xtype, _np_ptr(xbuf), nelems, None if xv is None else _np_ptr(xv)), "fill",
           (T.NC_NOERR,))


def dev_fill(xtype, dx, nelems, xvalue=None, stream=None):
    xv = None if xvalue is None else np.frombuffer(bytes(xvalue) + b"\0" * 8, np.uint8).copy()
    _check(lib().pncx_dev_fill(xtype, _dptr(dx), nelems, None if xv is None else _np_ptr(xv),
                               _stream_ptr(stream)), "dev_fill", (T.NC_NOERR,))


def _offs(vals):
    a = np.ascontiguousarray(np.asarray(vals, dtype=np.int64))
    return a, ctypes.c_void_p(a.ctypes.data)


def putn_imap(cdf_ver, xtype, xbuf, ibuf, count, imap, itype, fillp=None):
    """varm put: ibuf laid out by imap[] (elements), xbuf contiguous
    (create_imaptype.c + ncmpio_util.c:654-765, fused on the GPU)."""
    c, cp = _offs(count)
    m, mp = _offs(imap)
    fb = None if fillp is None else np.frombuffer(bytes(fillp) + b"\0" * 8, np.uint8).copy()
    return _check(lib().pncx_putn_imap(cdf_ver, xtype, _np_ptr(xbuf), _np_ptr(ibuf), len(c), cp, mp, itype,
                                       None if fb is None else _np_ptr(fb)), "putn_imap")


def getn_imap(cdf_ver, xtype, xbuf, ibuf, count, imap, itype):
    c, cp = _offs(count)
    m, mp = _offs(imap)
    return _check(lib().pncx_getn_imap(cdf_ver, xtype, _np_ptr(xbuf), _np_ptr(ibuf), len(c), cp, mp, itype),
                  "getn_imap")


def dev_putn_imap(cdf_ver, xtype, dx, di, count, imap, itype, fillp=None, dstatus=None, stream=None):
    c, cp = _offs(count)
    m, mp = _offs(imap)
    fb = None if fillp is None else np.frombuffer(bytes(fillp) + b"\0" * 8, np.uint8).copy()
    _check(lib().pncx_dev_putn_imap(cdf_ver, xtype, _dptr(dx), _dptr(di), len(c), cp, mp, itype,
                                    None if fb is None else _np_ptr(fb),
                                    None if dstatus is None else _dptr(dstatus), _stream_ptr(stream)),
           "dev_putn_imap", (T.NC_NOERR,))


def dev_getn_imap(cdf_ver, xtype, dx, di, count, imap, itype, dstatus=None, stream=None):
    c, cp = _offs(count)
    m, mp = _offs(imap)
    _check(lib().pncx_dev_getn_imap(cdf_ver, xtype, _dptr(dx), _dptr(di), len(c), cp, mp, itype,
                                    None if dstatus is None else _dptr(dstatus), _stream_ptr(stream)),
           "dev_getn_imap", (T.NC_NOERR,))


class DType:
    """A committed derived user-buffer datatype (pncx_type_commit): runs of
    blocklen[i] elements of itype at byte displacement disp[i], in pack
    order, one copy every `extent` bytes -- the flattened typemap of an MPI
    derived buftype (dtype_decode.c:628-694)."""

    def __init__(self, itype, disp, blocklen, extent):
        d, dp = _offs(disp)
        b, bp = _offs(blocklen)
        h = ctypes.c_void_p()
        _check(lib().pncx_type_commit(itype, len(d), dp, bp, extent, ctypes.byref(h)), "type_commit",
               (T.NC_NOERR,))
        self.handle = h
        self.itype = itype

    def inq(self):
        it, n, ext, lay = ctypes.c_int(), ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_int()
        _check(lib().pncx_type_inq(self.handle, ctypes.byref(it), ctypes.byref(n), ctypes.byref(ext),
                                   ctypes.byref(lay)), "type_inq", (T.NC_NOERR,))
        return {"itype": it.value, "nelems": n.value, "extent": ext.value, "layout": lay.value}

    def free(self):
        if self.handle:
            lib().pncx_type_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _fill_arg(fillp):
    fb = None if fillp is None else np.frombuffer(bytes(fillp) + b"\0" * 8, np.uint8).copy()
    return fb, (None if fb is None else _np_ptr(fb))


def putn_flex(cdf_ver, xtype, xbuf, buf, count, imap, bufcount, dtype, fillp=None, base=0):
    """put with a derived buftype: `buf` (numpy bytes) holds bufcount copies
    of dtype starting `base` bytes in (displacements may be negative)."""
    c, cp = _offs(count)
    mp = None if imap is None else _offs(imap)
    fb, fbp = _fill_arg(fillp)
    return _check(lib().pncx_putn_flex(cdf_ver, xtype, _np_ptr(xbuf), ctypes.c_void_p(buf.ctypes.data + base),
                                       len(c), cp, None if mp is None else mp[1], bufcount, dtype.handle, fbp),
                  "putn_flex")


def getn_flex(cdf_ver, xtype, xbuf, buf, count, imap, bufcount, dtype, base=0):
    c, cp = _offs(count)
    mp = None if imap is None else _offs(imap)
    return _check(lib().pncx_getn_flex(cdf_ver, xtype, _np_ptr(xbuf), ctypes.c_void_p(buf.ctypes.data + base),
                                       len(c), cp, None if mp is None else mp[1], bufcount, dtype.handle),
                  "getn_flex")


def dev_putn_flex(cdf_ver, xtype, dx, dbuf, count, imap, bufcount, dtype, fillp=None, dstatus=None,
                  stream=None, base=0):
    c, cp = _offs(count)
    mp = None if imap is None else _offs(imap)
    fb, fbp = _fill_arg(fillp)
    _check(lib().pncx_dev_putn_flex(cdf_ver, xtype, _dptr(dx), ctypes.c_void_p(dbuf.data_ptr() + base), len(c),
                                    cp, None if mp is None else mp[1], bufcount, dtype.handle, fbp,
                                    None if dstatus is None else _dptr(dstatus), _stream_ptr(stream)),
           "dev_putn_flex", (T.NC_NOERR,))


def dev_getn_flex(cdf_ver, xtype, dx, dbuf, count, imap, bufcount, dtype, dstatus=None, stream=None, base=0):
    c, cp = _offs(count)
    mp = None if imap is None else _offs(imap)
    _check(lib().pncx_dev_getn_flex(cdf_ver, xtype, _dptr(dx), ctypes.c_void_p(dbuf.data_ptr() + base), len(c),
                                    cp, None if mp is None else mp[1], bufcount, dtype.handle,
                                    None if dstatus is None else _dptr(dstatus), _stream_ptr(stream)),
           "dev_getn_flex", (T.NC_NOERR,))


def batch(segs):
    """Host-buffer batch: segs = list of dicts with dir, cdf_ver, xtype,
    itype, nelems, xbuf, ibuf (numpy), fill (bytes or None).  Returns the
    per-segment status list."""
    arr = (Seg * len(segs))()
    keep = []
    for k, s in enumerate(segs):
        fb = None
        if s.get("fill") is not None:
            fb = np.frombuffer(bytes(s["fill"]) + b"\0" * 8, np.uint8).copy()
            keep.append(fb)
        arr[k] = Seg(s["dir"], s.get("cdf_ver", 5), s["xtype"], s["itype"], s["nelems"],
                     s["xbuf"].ctypes.data, s["ibuf"].ctypes.data,
                     None if fb is None else fb.ctypes.data)
    st = (ctypes.c_int * len(segs))()
    rc = lib().pncx_batch(arr, len(segs), st)
    if rc not in (T.NC_NOERR, T.NC_ERANGE, T.NC_EBADTYPE, T.NC_ECHAR):
        raise PncxError(rc, "batch")
    return list(st)


# -------------------------------------------------------------- device side
# the HIP runtime's per-thread stream handle (hip_runtime_api.h: hipStreamPerThread)
STREAM_PER_THREAD = 2


def _stream_ptr(stream):
    """A torch stream, None (torch's current stream) or a raw hipStream_t value."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


def _dptr(t):
    assert t.is_cuda and t.is_contiguous()
    return ctypes.c_void_p(t.data_ptr())


def dev_in_swapn(t, nelems, esize, stream=None):
    """In-place swap of an HBM tensor (the config-2/5 hot kernel)."""
    _check(lib().pncx_dev_in_swapn(_dptr(t), nelems, esize, _stream_ptr(stream)), "dev_in_swapn",
           (T.NC_NOERR,))


def dev_swapn(dst, src, nelems, esize, stream=None):
    _check(lib().pncx_dev_swapn(_dptr(dst), _dptr(src), nelems, esize, _stream_ptr(stream)),
           "dev_swapn", (T.NC_NOERR,))


def dev_putn(cdf_ver, xtype, dx, di, nelems, itype, fillp=None, dstatus=None, stream=None):
    fb = None if fillp is None else np.frombuffer(bytes(fillp) + b"\0" * 8, np.uint8).copy()
    _check(lib().pncx_dev_putn(cdf_ver, xtype, _dptr(dx), _dptr(di), nelems, itype,
                               None if fb is None else _np_ptr(fb),
                               None if dstatus is None else _dptr(dstatus), _stream_ptr(stream)),
           "dev_putn", (T.NC_NOERR,))


def dev_getn(cdf_ver, xtype, dx, di, nelems, itype, dstatus=None, stream=None):
    _check(lib().pncx_dev_getn(cdf_ver, xtype, _dptr(dx), _dptr(di), nelems, itype,
                               None if dstatus is None else _dptr(dstatus), _stream_ptr(stream)),
           "dev_getn", (T.NC_NOERR,))


def _dev_segs(segs):
    arr = (Seg * len(segs))()
    keep = []
    for k, s in enumerate(segs):
        fb = None
        if s.get("fill") is not None:
            fb = np.frombuffer(bytes(s["fill"]) + b"\0" * 8, np.uint8).copy()
            keep.append(fb)
        arr[k] = Seg(s["dir"], s.get("cdf_ver", 5), s["xtype"], s["itype"], s["nelems"],
                     s["xbuf"].data_ptr(), s["ibuf"].data_ptr(),
                     None if fb is None else fb.ctypes.data)
    return arr, keep


def dev_batch_async(segs, dstatus, stream=None):
    """pncx_dev_batch_async: the statuses land in the int32 CUDA tensor
    `dstatus` (NC_ERANGE words) once the stream gets there; returns the
    call's code (the fill values are copied during the call)."""
    arr, keep = _dev_segs(segs)
    return lib().pncx_dev_batch_async(arr, len(segs), _dptr(dstatus), _stream_ptr(stream))


def dev_batch(segs, stream=None):
    """Device batch: like ``batch`` but xbuf/ibuf are CUDA tensors."""
    arr = (Seg * len(segs))()
    keep = []
    for k, s in enumerate(segs):
        fb = None
        if s.get("fill") is not None:
            fb = np.frombuffer(bytes(s["fill"]) + b"\0" * 8, np.uint8).copy()
            keep.append(fb)
        arr[k] = Seg(s["dir"], s.get("cdf_ver", 5), s["xtype"], s["itype"], s["nelems"],
                     s["xbuf"].data_ptr(), s["ibuf"].data_ptr(),
                     None if fb is None else fb.ctypes.data)
    st = (ctypes.c_int * len(segs))()
    rc = lib().pncx_dev_batch(arr, len(segs), st, _stream_ptr(stream))
    if rc not in (T.NC_NOERR, T.NC_ERANGE, T.NC_EBADTYPE, T.NC_ECHAR):
        raise PncxError(rc, "dev_batch")
    return list(st)
