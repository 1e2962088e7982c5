"""The reference's CDL fixture src/utils/ncmpigen/c0.cdl as a file-level pin
(GPU).  Its schema, attributes and data (tests/golden/c0_cdl.json, made by
tests/golden/make_c0.py) are written through the MI355X path as a CDF-1
file -- every numeric variable from a double buffer, so each value crosses
the double -> NC_<type> conversion at the type limits c0.cdl chose
(-32768s, 2147483647, +-1e+36f, +-1e+308) -- then:

  * an independent reader (scipy.io.netcdf_file) must see every dimension,
    attribute and variable value exactly as CDL types them (ncmpigen's
    semantics: a char variable's strings fill rows of its last dimension);
  * reading each numeric variable back through the GPU get path into every
    internal type must give the element values of a numpy restatement of
    the reference's range rules (NCX_GET1I / GETF_CheckBND, ncx.m4:503-598):
    out-of-range elements hold the internal type's fill and the call
    returns NC_ERANGE.

No oracle is involved: the expectations come from the CDL text and numpy.
"""
import json
import math
import os

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N

pytestmark = pytest.mark.gpu

FIX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c0_cdl.json")))
NUMERIC_ITYPES = [T.ITYPE_SCHAR, T.ITYPE_UCHAR, T.ITYPE_SHORT, T.ITYPE_USHORT, T.ITYPE_INT, T.ITYPE_UINT,
                  T.ITYPE_LONG, T.ITYPE_FLOAT, T.ITYPE_DOUBLE, T.ITYPE_LONGLONG, T.ITYPE_ULONGLONG]
FLT_MAX = float(np.finfo(np.float32).max)


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


def shape_of(var, nrec):
    return [nrec if FIX["dims"][d][1] == 0 else FIX["dims"][d][1] for d in var["dims"]]


def char_bytes(var, strings):
    """ncmpigen: a 1-D char variable is the concatenated text (padded with
    NULs to a fixed dimension); otherwise every string is padded to a
    multiple of the last dimension and the rows follow one another"""
    if len(var["dims"]) <= 1:
        b = b"".join(s.encode("latin1") for s in strings)
        ln = FIX["dims"][var["dims"][0]][1] if var["dims"] else 1
        return b + b"\0" * (ln - len(b)) if ln > len(b) else b
    last = FIX["dims"][var["dims"][-1]][1]
    out = b""
    for s in strings:
        b = s.encode("latin1")
        out += b + b"\0" * ((-len(b)) % last if b else last)
    return out


def expected_typed(var):
    d = FIX["data"][var["name"]]
    if var["xtype"] == T.NC_CHAR:
        return np.frombuffer(char_bytes(var, d["text"]), np.uint8)
    return np.array(d["numbers"], dtype=np.float64).astype(T.XTYPE_NP[var["xtype"]])


def nrecs():
    n = 0
    for v in FIX["vars"]:
        if v["dims"] and FIX["dims"][v["dims"][0]][1] == 0 and v["name"] in FIX["data"]:
            per = int(np.prod(shape_of(v, 1)))
            n = max(n, expected_typed(v).size // per)
    return n


def write_c0(path):
    err, ncid = N.create(path, 0)
    assert err == 0
    for name, ln in FIX["dims"]:
        assert N.def_dim(ncid, name, ln)[0] == 0
    ids = {}
    for v in FIX["vars"]:
        err, ids[v["name"]] = N.def_var(ncid, v["name"], v["xtype"], v["dims"])
        assert err == 0, v["name"]
    for a in FIX["atts"]:
        vid = N.NC_GLOBAL if a["var"] == "" else ids[a["var"]]
        if a["xtype"] == T.NC_CHAR:
            assert N.put_att_text(ncid, vid, a["name"], "".join(a["values"]).encode("latin1")) == 0
        else:
            arr = np.array(a["values"], dtype=np.float64).astype(T.XTYPE_NP[a["xtype"]])
            assert N.put_att(ncid, vid, a["name"], a["xtype"], arr) == 0, a["name"]
    assert N.enddef(ncid) == 0
    nr = nrecs()
    for v in FIX["vars"]:
        if v["name"] not in FIX["data"]:
            continue                            # c213: commented out in c0.cdl
        shp = shape_of(v, nr)
        if v["xtype"] == T.NC_CHAR:
            buf = expected_typed(v)
            assert N.put_var(ncid, ids[v["name"]], buf, [0] * len(shp), shp, itype=T.ITYPE_CHAR) == 0, v["name"]
        else:
            buf = np.array(FIX["data"][v["name"]]["numbers"], dtype=np.float64)
            st = N.put_var(ncid, ids[v["name"]], buf, [0] * len(shp) if shp else None, shp if shp else None)
            assert st == 0, (v["name"], st)
    assert N.close(ncid) == 0
    return nr


def test_c0_independent_reader(gpu, tmp_path):
    sio = pytest.importorskip("scipy.io")
    p = str(tmp_path / "c0.nc")
    nr = write_c0(p)
    assert nr == 2
    # The last record ends with cr33's 9 bytes: like the reference, the
    # library does not write the last record's padding (ncmpio_close.c
    # never extends a file), while scipy reads whole padded records.  It
    # reads a copy with zero bytes appended.
    q = str(tmp_path / "c0_scipy.nc")
    open(q, "wb").write(open(p, "rb").read() + b"\0" * 8)
    f = sio.netcdf_file(q, "r", mmap=False)
    try:
        for name, ln in FIX["dims"]:
            assert f.dimensions[name] == (None if ln == 0 else ln), name
        for a in FIX["atts"]:
            got = (f._attributes if a["var"] == "" else f.variables[a["var"]]._attributes)[a["name"]]
            if a["xtype"] == T.NC_CHAR:
                assert got == "".join(a["values"]).encode("latin1"), a["name"]
            else:
                exp = np.array(a["values"], dtype=np.float64).astype(T.XTYPE_NP[a["xtype"]])
                assert np.asarray(got).dtype.itemsize == exp.dtype.itemsize, a["name"]
                assert np.asarray(got).tobytes() == exp.astype(np.asarray(got).dtype).tobytes(), a["name"]
        for v in FIX["vars"]:
            if v["name"] not in FIX["data"]:
                continue
            got = f.variables[v["name"]].data
            exp = expected_typed(v)
            if v["xtype"] == T.NC_CHAR:
                assert np.asarray(got).tobytes() == exp.tobytes(), v["name"]
            else:
                assert np.asarray(got).reshape(-1).astype(exp.dtype).tobytes() == exp.tobytes(), v["name"]
    finally:
        f.close()


def expect_get(xvals, xtype, itype):
    """numpy restatement of NCX_GET1I / GETF_CheckBND for these values"""
    dt = np.dtype(T.ITYPE_NP[itype])
    out = np.empty(xvals.size, dt)
    bad = False
    is_float_x = xtype in (T.NC_FLOAT, T.NC_DOUBLE)
    for k, x in enumerate(xvals.tolist()):
        if dt.kind == "f":
            if dt.itemsize == 4 and xtype == T.NC_DOUBLE and abs(x) > FLT_MAX:
                bad, out[k] = True, T.ITYPE_FILL[itype]
            else:
                out[k] = x
            continue
        info = np.iinfo(dt)
        v = math.trunc(x) if is_float_x else int(x)
        lo, hi = (info.min, info.max)
        if (x > hi or x < lo) if is_float_x else (v > hi or v < lo):
            bad, out[k] = True, T.ITYPE_FILL[itype]
        else:
            out[k] = v
    return out, bad


def test_c0_cross_type_gets(gpu, tmp_path):
    p = str(tmp_path / "c0.nc")
    nr = write_c0(p)
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    try:
        for varid, v in enumerate(FIX["vars"]):
            if v["xtype"] == T.NC_CHAR or v["name"] not in FIX["data"]:
                continue
            xvals = expected_typed(v)
            shp = shape_of(v, nr)
            for it in NUMERIC_ITYPES:
                out = np.zeros(xvals.size, T.ITYPE_NP[it])
                st = N.get_var(ncid, varid, out, [0] * len(shp) if shp else None, shp if shp else None, itype=it)
                exp, bad = expect_get(xvals, v["xtype"], it)
                assert st == (T.NC_ERANGE if bad else 0), (v["name"], T.INAME[it], st)
                assert out.tobytes() == exp.tobytes(), (v["name"], T.INAME[it], out, exp)
    finally:
        N.close(ncid)
