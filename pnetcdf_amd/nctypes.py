"""NetCDF type metadata shared by the host mirror, tests and bench.

Constants mirror ``include/pncx.h`` (which cites src/include/pnetcdf.h.in:66-114
and src/drivers/common/convert_swap.m4:218-245 of the reference).
"""
import numpy as np

# external types (pnetcdf.h.in:66-83)
NC_BYTE, NC_CHAR, NC_SHORT, NC_INT, NC_FLOAT, NC_DOUBLE = 1, 2, 3, 4, 5, 6
NC_UBYTE, NC_USHORT, NC_UINT, NC_INT64, NC_UINT64 = 7, 8, 9, 10, 11

NC_NOERR, NC_EINVAL, NC_EBADTYPE, NC_ECHAR, NC_ERANGE, NC_ENOMEM = 0, -36, -45, -56, -60, -61
PNCX_EDEVICE = -1900
NC_EMULTITYPES, NC_EIOMISMATCH = -208, -209   # pnetcdf.h.in:629-630

# internal types (enum pncx_itype)
ITYPE_SCHAR, ITYPE_UCHAR, ITYPE_SHORT, ITYPE_USHORT, ITYPE_INT, ITYPE_UINT = 1, 2, 3, 4, 5, 6
ITYPE_LONG, ITYPE_FLOAT, ITYPE_DOUBLE, ITYPE_LONGLONG, ITYPE_ULONGLONG, ITYPE_CHAR = 7, 8, 9, 10, 11, 12

PNCX_PUT, PNCX_GET = 1, 2

XTYPES = {
    "byte": NC_BYTE, "ubyte": NC_UBYTE, "short": NC_SHORT, "ushort": NC_USHORT,
    "int": NC_INT, "uint": NC_UINT, "float": NC_FLOAT, "double": NC_DOUBLE,
    "int64": NC_INT64, "uint64": NC_UINT64,
}
NUMERIC_XTYPES = [NC_BYTE, NC_UBYTE, NC_SHORT, NC_USHORT, NC_INT, NC_UINT,
                  NC_FLOAT, NC_DOUBLE, NC_INT64, NC_UINT64]

ITYPES = {
    "schar": ITYPE_SCHAR, "uchar": ITYPE_UCHAR, "short": ITYPE_SHORT,
    "ushort": ITYPE_USHORT, "int": ITYPE_INT, "uint": ITYPE_UINT,
    "long": ITYPE_LONG, "float": ITYPE_FLOAT, "double": ITYPE_DOUBLE,
    "longlong": ITYPE_LONGLONG, "ulonglong": ITYPE_ULONGLONG,
}
NUMERIC_ITYPES = list(ITYPES.values())

# native numpy dtype of each external type's value (host byte order)
XTYPE_NP = {
    NC_BYTE: np.int8, NC_CHAR: np.uint8, NC_UBYTE: np.uint8, NC_SHORT: np.int16,
    NC_USHORT: np.uint16, NC_INT: np.int32, NC_UINT: np.uint32,
    NC_FLOAT: np.float32, NC_DOUBLE: np.float64, NC_INT64: np.int64,
    NC_UINT64: np.uint64,
}
# big-endian on-disk dtype
XTYPE_BE = {k: np.dtype(v).newbyteorder(">") for k, v in XTYPE_NP.items()}

ITYPE_NP = {
    ITYPE_SCHAR: np.int8, ITYPE_UCHAR: np.uint8, ITYPE_SHORT: np.int16,
    ITYPE_USHORT: np.uint16, ITYPE_INT: np.int32, ITYPE_UINT: np.uint32,
    ITYPE_LONG: np.int64, ITYPE_FLOAT: np.float32, ITYPE_DOUBLE: np.float64,
    ITYPE_LONGLONG: np.int64, ITYPE_ULONGLONG: np.uint64, ITYPE_CHAR: np.uint8,
}

XNAME = {v: k for k, v in XTYPES.items()}
XNAME[NC_CHAR] = "char"
INAME = {v: k for k, v in ITYPES.items()}
INAME[ITYPE_CHAR] = "char"


def xlen(xtype):
    return np.dtype(XTYPE_NP[xtype]).itemsize


def ilen(itype):
    return np.dtype(ITYPE_NP[itype]).itemsize


# default fill values of external types (pnetcdf.h.in:104-114), native value
XTYPE_FILL = {
    NC_BYTE: -127, NC_CHAR: 0, NC_SHORT: -32767, NC_INT: -2147483647,
    NC_FLOAT: np.float32(9.9692099683868690e+36), NC_DOUBLE: 9.9692099683868690e+36,
    NC_UBYTE: 255, NC_USHORT: 65535, NC_UINT: 4294967295,
    NC_INT64: -9223372036854775806, NC_UINT64: 18446744073709551614,
}
# get-side fill per internal type (ncx.m4:97-111; long -> NC_FILL_INT)
ITYPE_FILL = {
    ITYPE_SCHAR: -127, ITYPE_UCHAR: 255, ITYPE_SHORT: -32767, ITYPE_USHORT: 65535,
    ITYPE_INT: -2147483647, ITYPE_UINT: 4294967295, ITYPE_LONG: -2147483647,
    ITYPE_FLOAT: np.float32(9.9692099683868690e+36), ITYPE_DOUBLE: 9.9692099683868690e+36,
    ITYPE_LONGLONG: -9223372036854775806, ITYPE_ULONGLONG: 18446744073709551614,
}


def fill_bytes(xtype, value=None):
    """Native-order bytes of a fill value of xtype (what ncmpio_inq_var_fill
    hands to putn, ncmpio_util.c:705-711)."""
    v = XTYPE_FILL[xtype] if value is None else value
    return np.array([v], dtype=XTYPE_NP[xtype]).tobytes()


def need_convert(fmt, xtype, itype):
    """ncmpii_need_convert (convert_swap.m4:85-116)."""
    if xtype == NC_CHAR:
        return 0
    if fmt < 5 and xtype == NC_BYTE and itype == ITYPE_UCHAR:
        return 0
    if itype == ITYPE_LONG:
        itype = ITYPE_LONGLONG
    same = {(NC_BYTE, ITYPE_SCHAR), (NC_SHORT, ITYPE_SHORT), (NC_INT, ITYPE_INT),
            (NC_FLOAT, ITYPE_FLOAT), (NC_DOUBLE, ITYPE_DOUBLE), (NC_UBYTE, ITYPE_UCHAR),
            (NC_USHORT, ITYPE_USHORT), (NC_UINT, ITYPE_UINT), (NC_INT64, ITYPE_LONGLONG),
            (NC_UINT64, ITYPE_ULONGLONG)}
    return 0 if (xtype, itype) in same else 1
