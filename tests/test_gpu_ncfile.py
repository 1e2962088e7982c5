"""File-level parity on the GPU: data written and read through the HIP
conversion path land in the file exactly where and how the reference puts
them.

Expected file bytes come from the pinned oracle (conversion) and from numpy
big-endian encoding at offsets computed by the independent header parser
(tests/cdfparse.py); the reference-written tests/golden/tst_file.nc
(src/utils/ncmpidiff) is reproduced byte for byte.
"""
import os

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N
from tests import cdfparse
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


def _raw(p):
    return open(p, "rb").read()


def _var_bytes(raw, h, name, rec=None, nbytes=None):
    v = [x for x in h["vars"] if x["name"] == name][0]
    off = v["begin"] + (rec * h["recsize"] if rec is not None else 0)
    return raw[off:off + (nbytes if nbytes is not None else v["vsize"])]


def test_tst_file_full_byte_parity(gpu, tmp_path):
    """ncmpidiff fixture: same schema + same values -> identical 800 bytes"""
    ref = _raw(os.path.join(GOLD, "tst_file.nc"))
    h = cdfparse.parse_cdf(ref)
    fix = np.frombuffer(_var_bytes(ref, h, "fix_var"), ">f4").astype(np.float32)
    recs = [np.frombuffer(_var_bytes(ref, h, "rec_var", r, 48), ">f4").astype(np.float32) for r in range(2)]
    p = str(tmp_path / "t.nc")
    err, ncid = N.create(p, 0)
    N.def_dim(ncid, "time", N.NC_UNLIMITED)
    N.def_dim(ncid, "Y", 4)
    N.def_dim(ncid, "X", 12)
    N.put_att_text(ncid, N.NC_GLOBAL, "history", "Mon Aug 13 21:27:48 2018")
    N.def_var(ncid, "rec_var", T.NC_FLOAT, [0, 2])
    N.def_var(ncid, "fix_var", T.NC_FLOAT, [1, 2])
    assert N.enddef(ncid) == 0
    assert N.put_var(ncid, 1, fix) == 0
    assert N.put_var(ncid, 0, np.stack(recs), [0, 0], [2, 12]) == 0
    assert N.close(ncid) == 0
    assert _raw(p) == ref
    # and read back through the get path
    err, ncid = N.open(p)
    o = np.zeros((2, 12), np.float64)
    assert N.get_var(ncid, 0, o) == 0
    assert np.array_equal(o, np.stack(recs).astype(np.float64))
    assert N.close(ncid) == 0


ITYPES_FOR = {
    T.NC_BYTE: [T.ITYPE_SCHAR, T.ITYPE_INT, T.ITYPE_DOUBLE],
    T.NC_SHORT: [T.ITYPE_SHORT, T.ITYPE_FLOAT, T.ITYPE_LONGLONG],
    T.NC_INT: [T.ITYPE_INT, T.ITYPE_DOUBLE, T.ITYPE_SHORT],
    T.NC_FLOAT: [T.ITYPE_FLOAT, T.ITYPE_DOUBLE, T.ITYPE_INT],
    T.NC_DOUBLE: [T.ITYPE_DOUBLE, T.ITYPE_FLOAT, T.ITYPE_LONGLONG],
    T.NC_UBYTE: [T.ITYPE_UCHAR, T.ITYPE_INT],
    T.NC_USHORT: [T.ITYPE_USHORT, T.ITYPE_DOUBLE],
    T.NC_UINT: [T.ITYPE_UINT, T.ITYPE_LONGLONG],
    T.NC_INT64: [T.ITYPE_LONGLONG, T.ITYPE_DOUBLE, T.ITYPE_INT],
    T.NC_UINT64: [T.ITYPE_ULONGLONG, T.ITYPE_FLOAT],
}


@pytest.mark.parametrize("xt", T.NUMERIC_XTYPES, ids=[T.XNAME[x] for x in T.NUMERIC_XTYPES])
def test_vara_all_types_vs_oracle(gpu, tmp_path, xt):
    """record and fixed variables of every external type, several internal
    types, random bits (incl. out-of-range values -> fill, NC_ERANGE): file
    bytes = oracle putn of the same buffer; get = oracle getn of the file"""
    ora = OracleConv()
    rng = np.random.default_rng(0xF11E + xt)
    p = str(tmp_path / "v.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "time", N.NC_UNLIMITED)
    N.def_dim(ncid, "y", 5)
    N.def_dim(ncid, "x", 9)
    its = ITYPES_FOR[xt]
    for k, it in enumerate(its):
        N.def_var(ncid, f"f{k}", xt, [1, 2])
        N.def_var(ncid, f"r{k}", xt, [0, 1, 2])
    assert N.enddef(ncid) == 0
    wrote = {}
    for k, it in enumerate(its):
        ib = np.frombuffer(rng.bytes(45 * 8), T.ITYPE_NP[it])[:45].copy()
        if T.ITYPE_NP[it] in (np.float32, np.float64):
            ib[np.isnan(ib)] = 1.5           # NaN payload cases are covered by the conversion tests
        exp_x, exp_st = ora.putn(5, xt, ib, it, T.fill_bytes(xt))
        st = N.put_var(ncid, 2 * k, ib, [0, 0], [5, 9], itype=it)
        assert st == exp_st, (T.INAME[it], N.strerror(st))
        st = N.put_var(ncid, 2 * k + 1, ib, [2, 0, 0], [1, 5, 9], itype=it)
        assert st == exp_st
        wrote[k] = (ib, exp_x)
    assert N.close(ncid) == 0
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    assert h["numrecs"] == 3
    xs = T.xlen(xt)
    for k, it in enumerate(its):
        ib, exp_x = wrote[k]
        assert _var_bytes(raw, h, f"f{k}", None, 45 * xs) == exp_x
        assert _var_bytes(raw, h, f"r{k}", 2, 45 * xs) == exp_x
    err, ncid = N.open(p)
    for k, it in enumerate(its):
        exp_i, exp_st = ora.getn(5, xt, wrote[k][1], it)
        out = np.zeros(45, T.ITYPE_NP[it])
        assert N.get_var(ncid, 2 * k + 1, out, [2, 0, 0], [1, 5, 9], itype=it) == exp_st
        assert out.tobytes() == exp_i.tobytes()
    assert N.close(ncid) == 0


def test_vars_varm_layouts(gpu, tmp_path):
    """strided file access (vars) and a transposed user buffer (varm imap)"""
    p = str(tmp_path / "m.nc")
    err, ncid = N.create(p, N.NC_64BIT_OFFSET)
    N.def_dim(ncid, "y", 6)
    N.def_dim(ncid, "x", 8)
    N.def_var(ncid, "d", T.NC_DOUBLE, [0, 1])
    N.def_var(ncid, "i", T.NC_INT, [0, 1])
    assert N.enddef(ncid) == 0
    full = np.arange(48, dtype=np.float64).reshape(6, 8) + 0.25
    assert N.put_var(ncid, 0, full) == 0
    sub = -np.arange(12, dtype=np.float64).reshape(3, 4)
    assert N.put_var(ncid, 0, sub, [0, 1], [3, 4], [2, 2]) == 0          # rows 0,2,4 cols 1,3,5,7
    exp = full.copy()
    exp[0:6:2, 1:8:2] = sub
    # varm: user buffer holds the (6, 8) block transposed, i.e. imap = (1, 6)
    t = np.ascontiguousarray((np.arange(48, dtype=np.int32).reshape(6, 8) * 3).T)
    assert N.put_var(ncid, 1, t, [0, 0], [6, 8], None, [1, 6]) == 0
    assert N.close(ncid) == 0
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    assert np.frombuffer(_var_bytes(raw, h, "d"), ">f8").reshape(6, 8).tolist() == exp.tolist()
    assert np.array_equal(np.frombuffer(_var_bytes(raw, h, "i"), ">i4").reshape(6, 8),
                          np.arange(48).reshape(6, 8) * 3)
    err, ncid = N.open(p)
    o = np.zeros((3, 4), np.float32)
    assert N.get_var(ncid, 0, o, [1, 0], [3, 4], [2, 2]) == 0
    assert np.array_equal(o, exp[1:6:2, 0:8:2].astype(np.float32))
    ot = np.zeros((8, 6), np.int64)
    assert N.get_var(ncid, 1, ot, [0, 0], [6, 8], None, [1, 6]) == 0
    assert np.array_equal(ot, (np.arange(48).reshape(6, 8) * 3).T)
    assert N.close(ncid) == 0


def test_erange_fill_value_on_put(gpu, tmp_path):
    """test/testcases/erange_fill.m4: out-of-range puts write the variable's
    _FillValue (else the type default) and return NC_ERANGE"""
    p = str(tmp_path / "e.nc")
    err, ncid = N.create(p, 0)
    N.def_dim(ncid, "x", 4)
    N.def_var(ncid, "a", T.NC_INT, [0])
    N.def_var(ncid, "b", T.NC_SHORT, [0])
    assert N.put_att(ncid, 0, "_FillValue", T.NC_INT, np.array([-5], np.int32)) == 0
    assert N.enddef(ncid) == 0
    d = np.array([1e300, 1.0, -3e10, 7.0])
    assert N.put_var(ncid, 0, d) == N.NC_ERANGE
    assert N.put_var(ncid, 1, np.array([40000.0, 2.0, -40000.0, 3.0], np.float32)) == N.NC_ERANGE
    err, nf, fv = N.inq_var_fill(ncid, 0, np.int32)
    assert fv == -5
    assert N.close(ncid) == 0
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    assert np.frombuffer(_var_bytes(raw, h, "a", None, 16), ">i4").tolist() == [-5, 1, -5, 7]
    assert np.frombuffer(_var_bytes(raw, h, "b", None, 8), ">i2").tolist() == [-32767, 2, -32767, 3]


def test_fill_mode_and_fill_var_rec(gpu, tmp_path):
    """ncmpio_fill.c: fixed variables filled at enddef in NC_FILL mode (default
    or _FillValue pattern); record variables only by fill_var_rec"""
    p = str(tmp_path / "f.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "t", N.NC_UNLIMITED)
    N.def_dim(ncid, "x", 1000)
    assert N.set_fill(ncid, N.NC_FILL) == (0, N.NC_NOFILL)
    N.def_var(ncid, "s", T.NC_SHORT, [1])
    N.def_var(ncid, "d", T.NC_DOUBLE, [1])
    N.def_var(ncid, "u", T.NC_UINT64, [1])
    N.def_var(ncid, "r", T.NC_FLOAT, [0, 1])
    assert N.def_var_fill(ncid, 1, 0, np.float64(-1.25)) == 0
    assert N.enddef(ncid) == 0
    assert N.fill_var_rec(ncid, 3, 1) == 0                              # fills record 1, numrecs -> 2
    assert N.inq_dim(ncid, 0)[2] == 2
    assert N.fill_var_rec(ncid, 0, 0) == N.NC_ENOTRECVAR
    assert N.close(ncid) == 0
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    assert _var_bytes(raw, h, "s", None, 2000) == b"\x80\x01" * 1000
    assert np.all(np.frombuffer(_var_bytes(raw, h, "d", None, 8000), ">f8") == -1.25)
    assert _var_bytes(raw, h, "u", None, 8000) == b"\xff" * 7 + b"\xfe" + (b"\xff" * 7 + b"\xfe") * 999
    assert _var_bytes(raw, h, "r", 1, 4000) == b"\x7c\xf0\x00\x00" * 1000
    # NOFILL file: fill_var_rec needs a per-variable fill
    err, ncid = N.create(str(tmp_path / "g.nc"), 0)
    N.def_dim(ncid, "t", N.NC_UNLIMITED)
    N.def_var(ncid, "r", T.NC_INT, [0])
    assert N.enddef(ncid) == 0
    assert N.fill_var_rec(ncid, 0, 0) == N.NC_ENOTFILL
    assert N.close(ncid) == 0


def test_wait_all_fill_change_after_redef(gpu, tmp_path):
    """iput -> wait_all -> redef + def_var_fill -> iput -> wait_all: the
    second flush's ERANGE elements carry the new _FillValue even though the
    request list (and its arena addresses) repeat, so the batch plan cache
    must not reuse the first fill.  File bytes against
    the oracle's putn with each fill (ncmpio_util.c:705-711 takes the fill
    from ncmpio_inq_var_fill per request)."""
    nel = 8192
    p = str(tmp_path / "fillchg.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", nel)
    N.def_var(ncid, "s", T.NC_SHORT, [0])
    N.def_var(ncid, "f", T.NC_FLOAT, [0])
    assert N.enddef(ncid) == 0
    rng = np.random.default_rng(5)
    bs = rng.uniform(-40000, 40000, nel).astype(np.float32)     # ~18% ERANGE into NC_SHORT
    bf = rng.standard_normal(nel).astype(np.float32)
    ora = OracleConv()
    for k, fv in enumerate((None, -555, 1234)):
        if fv is not None:
            assert N.redef(ncid) == 0
            assert N.def_var_fill(ncid, 0, 0, np.array([fv], np.int16)) == 0
            assert N.enddef(ncid) == 0
        reqs = [N.iput_var(ncid, 0, bs, [0], [nel])[1], N.iput_var(ncid, 1, bf, [0], [nel])[1]]
        err, st = N.wait_all(ncid, reqs)
        assert err == N.NC_ERANGE and st == [N.NC_ERANGE, 0]
        assert N.sync(ncid) == 0
        raw = _raw(p)
        h = cdfparse.parse_cdf(raw)
        fill = T.fill_bytes(T.NC_SHORT, fv)
        exp, so = ora.putn(5, T.NC_SHORT, bs, T.ITYPE_FLOAT, fill)
        assert so == T.NC_ERANGE
        assert _var_bytes(raw, h, "s", None, nel * 2) == exp, (k, fv)
    assert N.close(ncid) == 0


def test_pending_requests_across_redef(gpu, tmp_path):
    """ncmpio_redef (ncmpio_file_misc.c:80-108) accepts pending nonblocking
    requests.  iput + iget posted, redef adds a variable and a header-growing
    attribute, enddef moves the data, then wait_all: the put lands at the
    variable's new offset, the get reads the moved data, and the put's
    ERANGE elements carry the fill of POST time (the reference converts an
    iput when it is posted, ncmpio_i_getput.m4:300-303), not the
    _FillValue defined in between."""
    nel = 4096
    p = str(tmp_path / "pend.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", nel)
    N.def_var(ncid, "a", T.NC_SHORT, [0])
    N.def_var(ncid, "b", T.NC_INT, [0])
    assert N.enddef(ncid) == 0
    rng = np.random.default_rng(9)
    vb = rng.integers(-2**31, 2**31 - 1, nel, dtype=np.int32)
    assert N.put_var(ncid, 1, vb) == 0
    off_a0 = N.inq_varoffset(ncid, 0)[1]
    va = rng.uniform(-40000, 40000, nel).astype(np.float64)
    got = np.zeros(nel, np.int64)
    err, rp = N.iput_var(ncid, 0, va, [0], [nel])
    assert err == 0
    err, rg = N.iget_var(ncid, 1, got, [0], [nel])
    assert err == 0
    assert N.redef(ncid) == 0
    assert N.put_att_text(ncid, N.NC_GLOBAL, "pad", "z" * 3000) == 0
    N.def_var(ncid, "c", T.NC_DOUBLE, [0])
    assert N.def_var_fill(ncid, 0, 0, np.array([-77], np.int16)) == 0
    assert N.enddef(ncid) == 0
    assert N.inq_varoffset(ncid, 0)[1] > off_a0                # the data moved
    err, st = N.wait_all(ncid, [rp, rg])
    assert err == N.NC_ERANGE and st == [N.NC_ERANGE, 0]
    assert np.array_equal(got, vb.astype(np.int64))
    assert N.close(ncid) == 0
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    exp, _ = OracleConv().putn(5, T.NC_SHORT, va, T.ITYPE_DOUBLE, T.fill_bytes(T.NC_SHORT))
    assert _var_bytes(raw, h, "a", None, nel * 2) == exp
    assert _var_bytes(raw, h, "b", None, nel * 4) == vb.astype(">i4").tobytes()


def test_nonblocking_c4_batch(gpu, tmp_path):
    """config-4 shape: many iput_vara of mixed NC_SHORT / NC_FLOAT flushed by
    one wait_all (one batched conversion); statuses per request, NC_ERANGE
    only where a value is out of range; then iget back"""
    nvar, nel = 64, 4096
    p = str(tmp_path / "c4.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", nel)
    for v in range(nvar):
        N.def_var(ncid, f"v{v}", T.NC_SHORT if v % 2 == 0 else T.NC_FLOAT, [0])
    assert N.enddef(ncid) == 0
    rng = np.random.default_rng(0x5EED0004)
    bufs, reqs = [], []
    for v in range(nvar):
        if v % 2 == 0:
            b = rng.integers(-32768, 32767, nel, dtype=np.int16)
        else:
            b = rng.standard_normal(nel).astype(np.float32)
        if v == 6:
            b = rng.uniform(-40000, 40000, nel).astype(np.float32)    # short <- float, ~18% ERANGE
        bufs.append(b)
        err, rq = N.iput_var(ncid, v, b, [0], [nel])
        assert err == 0
        reqs.append(rq)
    err, st = N.wait_all(ncid, reqs)
    assert err == N.NC_ERANGE
    assert st[6] == N.NC_ERANGE and all(s == 0 for i, s in enumerate(st) if i != 6)
    assert N.close(ncid) == 0
    ora = OracleConv()
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    for v in range(nvar):
        xt = T.NC_SHORT if v % 2 == 0 else T.NC_FLOAT
        it = N.itype_of(bufs[v])
        exp, _ = ora.putn(5, xt, bufs[v], it, T.fill_bytes(xt))
        assert _var_bytes(raw, h, f"v{v}", None, nel * T.xlen(xt)) == exp, v
    err, ncid = N.open(p)
    outs = [np.zeros(nel, np.float64) for _ in range(nvar)]
    greqs = [N.iget_var(ncid, v, outs[v], [0], [nel])[1] for v in range(nvar)]
    err, st = N.wait_all(ncid, greqs)
    assert err == 0
    for v in range(nvar):
        xt = T.NC_SHORT if v % 2 == 0 else T.NC_FLOAT
        e, _ = ora.getn(5, xt, _var_bytes(raw, h, f"v{v}", None, nel * T.xlen(xt)), T.ITYPE_DOUBLE)
        assert outs[v].tobytes() == e.tobytes()
    assert N.close(ncid) == 0


def test_device_buffers(gpu, tmp_path):
    """put/get from HBM: conversion in HBM, packed bytes over PCIe once"""
    torch = gpu
    p = str(tmp_path / "dev.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "t", N.NC_UNLIMITED)
    N.def_dim(ncid, "x", 1 << 16)
    N.def_var(ncid, "r", T.NC_INT, [0, 1])
    N.def_var(ncid, "d", T.NC_DOUBLE, [1])
    assert N.enddef(ncid) == 0
    src = torch.arange(3 << 16, dtype=torch.float64, device="cuda").reshape(3, 1 << 16) - 70000.5
    assert N.put_var_dev(ncid, 0, src, [0, 0], [3, 1 << 16]) == 0
    dd = torch.randn(1 << 16, dtype=torch.float64, device="cuda")
    assert N.put_var_dev(ncid, 1, dd) == 0
    back = torch.empty(3, 1 << 16, dtype=torch.int64, device="cuda")
    assert N.get_var_dev(ncid, 0, back) == 0
    assert torch.equal(back, torch.trunc(src).to(torch.int64))
    dback = torch.empty(1 << 16, dtype=torch.float64, device="cuda")
    assert N.get_var_dev(ncid, 1, dback) == 0
    assert torch.equal(dback, dd)
    assert N.close(ncid) == 0
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    assert np.array_equal(np.frombuffer(_var_bytes(raw, h, "d", None, 8 << 16), ">f8"), dd.cpu().numpy())
    assert np.array_equal(np.frombuffer(_var_bytes(raw, h, "r", 2, 4 << 16), ">i4"),
                          np.trunc(src[2].cpu().numpy()).astype(np.int32))


def test_numeric_attributes(gpu, tmp_path):
    p = str(tmp_path / "att.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", 2)
    N.def_var(ncid, "v", T.NC_FLOAT, [0])
    assert N.put_att(ncid, N.NC_GLOBAL, "shorts", T.NC_SHORT, np.array([1, -2, 3], np.int32)) == 0
    assert N.put_att(ncid, 0, "range", T.NC_DOUBLE, np.array([0.5, 1e10], np.float32)) == 0
    assert N.put_att(ncid, 0, "big", T.NC_BYTE, np.array([1, 300], np.int32)) == N.NC_ERANGE
    assert N.put_att(ncid, 0, "u64", T.NC_UINT64, np.array([2**63 + 5], np.uint64)) == 0
    assert N.enddef(ncid) == 0
    assert N.close(ncid) == 0
    err, ncid = N.open(p)
    assert N.get_att(ncid, N.NC_GLOBAL, "shorts")[1].tolist() == [1, -2, 3]
    assert N.get_att(ncid, 0, "range")[1].tolist() == [0.5, np.float32(1e10)]
    assert N.get_att(ncid, 0, "big", np.int32)[1].tolist() == [1, -127]
    assert N.get_att(ncid, 0, "u64")[1].tolist() == [2**63 + 5]
    assert N.close(ncid) == 0
    h = cdfparse.parse_cdf(_raw(p))
    assert h["gatts"]["shorts"][0] == T.NC_SHORT


def test_redef_with_numeric_data(gpu, tmp_path):
    p = str(tmp_path / "rd.nc")
    err, ncid = N.create(p, 0)
    N.def_dim(ncid, "t", N.NC_UNLIMITED)
    N.def_dim(ncid, "x", 100)
    N.def_var(ncid, "a", T.NC_DOUBLE, [1])
    N.def_var(ncid, "r", T.NC_INT, [0, 1])
    assert N.enddef(ncid) == 0
    a = np.linspace(-1, 1, 100)
    r = np.arange(300, dtype=np.int32).reshape(3, 100)
    assert N.put_var(ncid, 0, a) == 0
    assert N.put_var(ncid, 1, r, [0, 0], [3, 100]) == 0
    assert N.redef(ncid) == 0
    assert N.set_fill(ncid, N.NC_FILL)[0] == 0
    N.def_var(ncid, "b", T.NC_SHORT, [1])
    N.def_var(ncid, "r2", T.NC_FLOAT, [0, 1])
    assert N._enddef(ncid, 0, 4096, 0, 0) == 0            # larger v_align: everything moves
    assert N.inq_varoffset(ncid, 0)[1] == 4096
    o = np.zeros(100)
    assert N.get_var(ncid, 0, o) == 0 and np.array_equal(o, a)
    orr = np.zeros((3, 100), np.int32)
    assert N.get_var(ncid, 1, orr, [0, 0], [3, 100]) == 0 and np.array_equal(orr, r)
    ob = np.zeros(100, np.int16)
    assert N.get_var(ncid, 2, ob) == 0 and np.all(ob == -32767)           # filled at enddef
    o2 = np.zeros((3, 100), np.float32)
    assert N.get_var(ncid, 3, o2, [0, 0], [3, 100]) == 0
    assert np.all(o2 == np.float32(9.9692099683868690e+36))               # existing records filled
    assert N.close(ncid) == 0


def test_large_variable_roundtrip(gpu, tmp_path):
    """a 256 MiB NC_DOUBLE variable through the host path and the device path"""
    torch = gpu
    n = 32 << 20
    p = str(tmp_path / "big.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", n)
    N.def_var(ncid, "a", T.NC_DOUBLE, [0])
    N.def_var(ncid, "b", T.NC_FLOAT, [0])
    assert N.enddef(ncid) == 0
    a = np.random.default_rng(3).standard_normal(n)
    assert N.put_var(ncid, 0, a) == 0
    t = torch.from_numpy(a).cuda()
    assert N.put_var_dev(ncid, 1, t) == 0
    o = np.empty(n)
    assert N.get_var(ncid, 0, o) == 0 and np.array_equal(o, a)
    ob = torch.empty(n, dtype=torch.float32, device="cuda")
    assert N.get_var_dev(ncid, 1, ob) == 0
    assert torch.equal(ob, t.float())
    assert N.close(ncid) == 0
    with open(p, "rb") as f:
        h = cdfparse.parse_cdf(f.read(4096))
        f.seek(h["vars"][0]["begin"] + 8 * (n - 4))
        assert np.array_equal(np.frombuffer(f.read(32), ">f8"), a[-4:])


def test_varn_numeric(gpu, tmp_path):
    """put_varn / get_varn of doubles into an NC_FLOAT variable: boxes packed
    in one buffer, one batched conversion, bytes = oracle putn per box"""
    ora = OracleConv()
    p = str(tmp_path / "vn.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "y", 40)
    N.def_dim(ncid, "x", 50)
    N.def_var(ncid, "f", T.NC_FLOAT, [0, 1])
    assert N.enddef(ncid) == 0
    starts = [[0, 0], [10, 5], [39, 49], [20, 0]]
    counts = [[3, 50], [7, 11], None, [10, 30]]
    sizes = [150, 77, 1, 300]
    rng = np.random.default_rng(9)
    buf = rng.standard_normal(sum(sizes)) * 1e3
    buf[7] = 1e300                                       # one ERANGE element
    assert N.put_varn(ncid, 0, starts, counts, buf) == N.NC_ERANGE
    back = np.zeros(sum(sizes), np.float64)
    assert N.get_varn(ncid, 0, starts, counts, back) == 0
    assert N.close(ncid) == 0
    exp, st = ora.putn(5, T.NC_FLOAT, buf, T.ITYPE_DOUBLE, T.fill_bytes(T.NC_FLOAT))
    assert st == N.NC_ERANGE
    e_back, _ = ora.getn(5, T.NC_FLOAT, exp, T.ITYPE_DOUBLE)
    assert back.tobytes() == e_back.tobytes()
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    f = np.frombuffer(_var_bytes(raw, h, "f", None, 40 * 50 * 4), ">f4").reshape(40, 50)
    e = np.frombuffer(exp, ">f4")
    assert f[0:3, :].tobytes() == e[:150].tobytes()
    assert f[10:17, 5:16].tobytes() == e[150:227].tobytes()
    assert f[39:40, 49:50].tobytes() == e[227:228].tobytes()      # slice: a scalar loses the byte order
    assert f[20:30, 0:30].tobytes() == e[228:].tobytes()


def test_bput_numeric(gpu, tmp_path):
    """buffered puts of doubles into NC_SHORT: converted at post (NC_ERANGE
    reported there), written at wait"""
    ora = OracleConv()
    p = str(tmp_path / "bp.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", 1000)
    N.def_var(ncid, "s", T.NC_SHORT, [0])
    assert N.enddef(ncid) == 0
    assert N.buffer_attach(ncid, 2000) == 0
    d = np.linspace(-50000, 50000, 1000)
    err, r1 = N.bput_var(ncid, 0, d[:500].copy(), [0], [500])
    assert err == N.NC_ERANGE and r1 >= 0
    err, r2 = N.bput_var(ncid, 0, d[500:].copy(), [500], [500])
    assert err == N.NC_ERANGE
    assert N.inq_buffer_usage(ncid) == (0, 2000)
    assert N.wait_all(ncid, [r1, r2]) == (0, [0, 0])
    assert N.buffer_detach(ncid) == 0
    assert N.close(ncid) == 0
    exp, _ = ora.putn(5, T.NC_SHORT, d, T.ITYPE_DOUBLE, T.fill_bytes(T.NC_SHORT))
    raw = _raw(p)
    h = cdfparse.parse_cdf(raw)
    assert _var_bytes(raw, h, "s", None, 2000) == exp
