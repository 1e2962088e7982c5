"""ctypes access to the reference-named ncx.h interface (include/pncx_ncx.h,
libpncx_ncmpii.so): ncmpix_{getn,pad_getn,putn,pad_putn}_<xtype>_<itype>,
the text/void byte copies and the header primitives.  Used by the tests;
the names, argument order and pointer-advance behaviour are the reference's
(src/drivers/include/ncx_h.m4:225-374)."""
import ctypes
import os

from . import nctypes as T
from . import pncx

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libpncx_ncmpii.so")

ITYPE_NAMES = [("schar", T.ITYPE_SCHAR), ("uchar", T.ITYPE_UCHAR), ("short", T.ITYPE_SHORT),
               ("ushort", T.ITYPE_USHORT), ("int", T.ITYPE_INT), ("uint", T.ITYPE_UINT), ("long", T.ITYPE_LONG),
               ("float", T.ITYPE_FLOAT), ("double", T.ITYPE_DOUBLE), ("longlong", T.ITYPE_LONGLONG),
               ("ulonglong", T.ITYPE_ULONGLONG)]
PADDED = [("NC_BYTE", T.NC_BYTE), ("NC_UBYTE", T.NC_UBYTE), ("NC_SHORT", T.NC_SHORT), ("NC_USHORT", T.NC_USHORT)]
UNPADDED = [("NC_INT", T.NC_INT), ("NC_UINT", T.NC_UINT), ("NC_FLOAT", T.NC_FLOAT), ("NC_DOUBLE", T.NC_DOUBLE),
            ("NC_INT64", T.NC_INT64), ("NC_UINT64", T.NC_UINT64)]

_lib = None


def lib():
    global _lib
    if _lib is None:
        pncx.lib()                                   # libpncx.so (and torch's HIP runtime) first
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def functions():
    """(name, op, xtype, itype, pad) of the 308 typed aggregate conversions"""
    out = []
    for xts, ops in ((PADDED, ("getn", "pad_getn", "putn", "pad_putn")), (UNPADDED, ("getn", "putn"))):
        for xname, xt in xts:
            for op in ops:
                for iname, it in ITYPE_NAMES:
                    out.append((f"ncmpix_{op}_{xname}_{iname}", op, xt, it, op.startswith("pad_")))
    return out


def call_get(name, xaddr, n, iaddr):
    """-> (status, bytes *xpp advanced)"""
    f = getattr(lib(), name)
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_longlong, ctypes.c_void_p]
    xp = ctypes.c_void_p(xaddr)
    st = f(ctypes.byref(xp), n, ctypes.c_void_p(iaddr))
    return st, (xp.value or 0) - xaddr


def call_put(name, xaddr, n, iaddr, faddr=None, text=False):
    f = getattr(lib(), name)
    f.restype = ctypes.c_int
    f.argtypes = ([ctypes.POINTER(ctypes.c_void_p), ctypes.c_longlong, ctypes.c_void_p] +
                  ([] if text else [ctypes.c_void_p]))
    xp = ctypes.c_void_p(xaddr)
    args = [ctypes.byref(xp), n, ctypes.c_void_p(iaddr)] + ([] if text else [ctypes.c_void_p(faddr)])
    st = f(*args)
    return st, (xp.value or 0) - xaddr
