"""ctypes front-end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / the timed CPU baseline.  The product
path (pnetcdf_amd) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    """Compile the oracle (gcc only; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "pncx_oracle.c")
        if (not os.path.exists(_LIB_PATH)
                or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_in_swapn.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int]
        L.orc_in_swapn.restype = None
        L.orc_need_convert.argtypes = [ctypes.c_int] * 3
        L.orc_need_swap.argtypes = [ctypes.c_int] * 2
        L.orc_getn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_longlong, ctypes.c_int]
        L.orc_putn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def in_swapn(buf, esize):
    """In place on a contiguous numpy array (any dtype); nelems = nbytes/esize."""
    assert buf.flags["C_CONTIGUOUS"]
    n = buf.nbytes // esize if esize > 0 else 0
    lib().orc_in_swapn(_ptr(buf), n, esize)
    return buf


def need_convert(fmt, xtype, itype):
    return lib().orc_need_convert(fmt, xtype, itype)


def need_swap(xtype, itype):
    return lib().orc_need_swap(xtype, itype)


def getn(cdf_ver, xtype, xbytes, itype, nelems=None):
    """external bytes (big-endian) -> (internal numpy array, status)"""
    from pnetcdf_amd import nctypes as T
    xs = T.xlen(xtype)
    xb = np.frombuffer(bytes(xbytes), dtype=np.uint8).copy()
    n = len(xb) // xs if nelems is None else nelems
    out = np.zeros(n, dtype=T.ITYPE_NP[itype])
    st = lib().orc_getn(cdf_ver, xtype, _ptr(xb), _ptr(out), n, itype)
    return out, st


def putn(cdf_ver, xtype, ibuf, itype, fill=None, xinit=None):
    """internal numpy array -> (external bytes, status).  fill: native-order
    bytes of the xtype fill value, or None for fillp == NULL.  xinit: prior
    content of the external buffer (matters only for NULL-fill cases)."""
    from pnetcdf_amd import nctypes as T
    ibuf = np.ascontiguousarray(ibuf, dtype=T.ITYPE_NP[itype])
    n = ibuf.size
    xs = T.xlen(xtype)
    if xinit is None:
        xb = np.zeros(n * xs, dtype=np.uint8)
    else:
        xb = np.frombuffer(bytes(xinit), dtype=np.uint8).copy()
    fb = None
    if fill is not None:
        fb = np.frombuffer(bytes(fill) + b"\0" * 8, dtype=np.uint8).copy()
    st = lib().orc_putn(cdf_ver, xtype, _ptr(xb), _ptr(ibuf), n, itype,
                        _ptr(fb) if fb is not None else None)
    return xb.tobytes(), st
