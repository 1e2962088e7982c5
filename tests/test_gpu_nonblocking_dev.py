"""Nonblocking requests whose user buffers live in HBM, mixed with host
requests in one wait_all (pncx_nc.c run_dir): the device requests convert
on the device between the user buffer and a device arena that crosses PCIe
with one copy; contiguous ones go through one pncx_dev_batch, varm and
derived-buftype ones get a fused launch and a status word each.  The
reference converts each request at post (iput, ncmpio_i_getput.m4:238-320)
or after the read (iget, ncmpio_wait.c:743-806); statuses are per request
and NC_ERANGE is not fatal (ncx.m4:2487-2488).

Every case checks per-request statuses and the file bytes (or the buffer
read back) against the oracle's putn/getn of the same values."""
import ctypes
import os

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N
from tests import cdfparse
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


def _offs(v):
    if v is None:
        return None, None
    a = np.ascontiguousarray(np.asarray(v, dtype=np.int64))
    return a, ctypes.c_void_p(a.ctypes.data)


def _ptr(buf):
    return ctypes.c_void_p(buf.data_ptr() if hasattr(buf, "data_ptr") else buf.ctypes.data)


def _post(fn, ncid, varid, buf, itype, start=None, count=None, stride=None, imap=None):
    keep = [_offs(x) for x in (start, count, stride, imap)]
    r = ctypes.c_int(N.NC_REQ_NULL)
    err = fn(ncid, varid, *[k[1] for k in keep], _ptr(buf), itype, ctypes.byref(r))
    return err, r.value


def iput(ncid, varid, buf, itype, **kw):
    return _post(N.lib().pncx_nc_iput_varm, ncid, varid, buf, itype, **kw)


def iget(ncid, varid, buf, itype, **kw):
    return _post(N.lib().pncx_nc_iget_varm, ncid, varid, buf, itype, **kw)


def bput(ncid, varid, buf, itype, **kw):
    return _post(N.lib().pncx_nc_bput_varm, ncid, varid, buf, itype, **kw)


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _var(raw, name):
    h = cdfparse.parse_cdf(raw)
    v = [x for x in h["vars"] if x["name"] == name][0]
    return raw[v["begin"]:v["begin"] + v["vsize"]]


def test_iget_dev_conversion_erange_mixed_with_host(torch_cuda, tmp_path):
    """iget NC_DOUBLE -> int32 into HBM with values out of int range
    (NC_ERANGE, fill), an iget of the same variable into a host buffer, and
    an iget NC_SHORT -> float into HBM, completed by one wait_all"""
    torch = torch_cuda
    ora = OracleConv()
    n = 4099
    rng = np.random.default_rng(7)
    d = rng.uniform(-1e3, 1e3, n)
    d[::11] = 3e10                                     # out of int range
    s = rng.integers(-32768, 32767, n).astype(np.int16)
    p = str(tmp_path / "g.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", n)
    N.def_var(ncid, "d", T.NC_DOUBLE, [0])
    N.def_var(ncid, "s", T.NC_SHORT, [0])
    assert N.enddef(ncid) == 0
    assert N.put_var(ncid, 0, d) == 0 and N.put_var(ncid, 1, s) == 0
    td = torch.zeros(n, dtype=torch.int32, device="cuda")
    hd = np.zeros(n, np.int32)
    ts = torch.zeros(n, dtype=torch.float32, device="cuda")
    e1, r1 = iget(ncid, 0, td, T.ITYPE_INT)
    e2, r2 = iget(ncid, 0, hd, T.ITYPE_INT)
    e3, r3 = iget(ncid, 1, ts, T.ITYPE_FLOAT)
    assert (e1, e2, e3) == (0, 0, 0)
    err, st = N.wait_all(ncid, [r1, r2, r3])
    xd = np.asarray(d, ">f8").tobytes()
    exp_i, exp_st = ora.getn(5, T.NC_DOUBLE, xd, T.ITYPE_INT)
    assert exp_st == T.NC_ERANGE
    assert st == [T.NC_ERANGE, T.NC_ERANGE, 0] and err == T.NC_ERANGE
    assert td.cpu().numpy().tobytes() == exp_i.tobytes()
    assert hd.tobytes() == exp_i.tobytes()
    exp_f, _ = ora.getn(5, T.NC_SHORT, np.asarray(s, ">i2").tobytes(), T.ITYPE_FLOAT)
    assert ts.cpu().numpy().tobytes() == exp_f.tobytes()
    assert N.close(ncid) == 0


def test_iput_varm_and_flex_dev_mixed_with_host(torch_cuda, tmp_path):
    """one wait_all over: a transposing iput_varm from HBM, a derived-buftype
    iput from HBM (every other int of a 2n buffer, into NC_SHORT with
    NC_ERANGE), the same two from host memory into twin variables, and a
    contiguous device iput; then iget of a derived buftype into HBM"""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    ny, nx = 37, 53
    rng = np.random.default_rng(11)
    full = rng.uniform(-100, 100, (ny, nx))
    tr = np.ascontiguousarray(full.T)                  # user buffer holds the transpose: imap (1, ny)
    n = ny * nx
    ints = rng.integers(-40000, 40000, 2 * n).astype(np.int32)
    dt = pncx.DType(T.ITYPE_INT, [0], [1], 8)          # vector: 1 int of every 2
    p = str(tmp_path / "m.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "y", ny)
    N.def_dim(ncid, "x", nx)
    for name, xt in (("vd", T.NC_DOUBLE), ("vh", T.NC_DOUBLE), ("fd", T.NC_SHORT), ("fh", T.NC_SHORT),
                     ("cd", T.NC_FLOAT)):
        N.def_var(ncid, name, xt, [0, 1])
    assert N.enddef(ncid) == 0
    keep = []
    ids = []
    dtr = _dev(torch, tr)
    keep.append(dtr)
    e, r = iput(ncid, 0, dtr, T.ITYPE_DOUBLE, start=[0, 0], count=[ny, nx], imap=[1, ny])
    assert e == 0
    ids.append(r)
    e, r = iput(ncid, 1, tr, T.ITYPE_DOUBLE, start=[0, 0], count=[ny, nx], imap=[1, ny])
    assert e == 0
    ids.append(r)
    dints = _dev(torch, ints)
    keep.append(dints)
    st = ctypes.c_int(N.NC_REQ_NULL)
    s0, c0 = _offs([0, 0]), _offs([ny, nx])
    e = N.lib().pncx_nc_iput_varm_flex(ncid, 2, s0[1], c0[1], None, None, _ptr(dints), n, dt.handle,
                                       ctypes.byref(st))
    assert e == 0
    ids.append(st.value)
    st2 = ctypes.c_int(N.NC_REQ_NULL)
    e = N.lib().pncx_nc_iput_varm_flex(ncid, 3, s0[1], c0[1], None, None, _ptr(ints), n, dt.handle,
                                       ctypes.byref(st2))
    assert e == 0
    ids.append(st2.value)
    fl = rng.standard_normal(n).astype(np.float32)
    dfl = _dev(torch, fl)
    keep.append(dfl)
    e, r = iput(ncid, 4, dfl, T.ITYPE_FLOAT, start=[0, 0], count=[ny, nx])
    assert e == 0
    ids.append(r)
    err, sts = N.wait_all(ncid, ids)
    assert sts == [0, 0, T.NC_ERANGE, T.NC_ERANGE, 0] and err == T.NC_ERANGE
    # iget of the derived buftype into HBM: the gaps must survive
    back = torch.full((2 * n,), -7, dtype=torch.int32, device="cuda")
    st3 = ctypes.c_int(N.NC_REQ_NULL)
    e = N.lib().pncx_nc_iget_varm_flex(ncid, 2, s0[1], c0[1], None, None, _ptr(back), n, dt.handle,
                                       ctypes.byref(st3))
    assert e == 0
    err, sts = N.wait_all(ncid, [st3.value])
    assert err == 0 and sts == [0]
    assert N.close(ncid) == 0
    dt.free()
    raw = open(p, "rb").read()
    exp_v, _ = ora.putn(5, T.NC_DOUBLE, full.reshape(-1), T.ITYPE_DOUBLE, T.fill_bytes(T.NC_DOUBLE))
    assert _var(raw, "vd") == exp_v and _var(raw, "vh") == exp_v
    exp_f, fst = ora.putn(5, T.NC_SHORT, ints[::2].copy(), T.ITYPE_INT, T.fill_bytes(T.NC_SHORT))
    assert fst == T.NC_ERANGE
    assert _var(raw, "fd")[:len(exp_f)] == exp_f and _var(raw, "fh")[:len(exp_f)] == exp_f
    exp_c, _ = ora.putn(5, T.NC_FLOAT, fl, T.ITYPE_FLOAT, T.fill_bytes(T.NC_FLOAT))
    assert _var(raw, "cd") == exp_c
    got = back.cpu().numpy()
    exp_i, _ = ora.getn(5, T.NC_SHORT, exp_f, T.ITYPE_INT)
    assert np.array_equal(got[::2], exp_i) and (got[1::2] == -7).all()


def test_one_byte_dev_iput_iget(torch_cuda, tmp_path):
    """NC_BYTE <-> schar (no conversion: a device copy) and NC_BYTE <- int
    (a conversion with NC_ERANGE), from and into HBM, CDF-2 and CDF-5"""
    torch = torch_cuda
    ora = OracleConv()
    n = 1000
    rng = np.random.default_rng(3)
    sc = rng.integers(-128, 127, n).astype(np.int8)
    iv = rng.integers(-300, 300, n).astype(np.int32)
    for fmt, cmode in ((2, N.NC_64BIT_OFFSET), (5, N.NC_64BIT_DATA)):
        p = str(tmp_path / f"b{fmt}.nc")
        err, ncid = N.create(p, cmode)
        N.def_dim(ncid, "x", n)
        N.def_var(ncid, "a", T.NC_BYTE, [0])
        N.def_var(ncid, "b", T.NC_BYTE, [0])
        assert N.enddef(ncid) == 0
        da, db = _dev(torch, sc), _dev(torch, iv)
        e1, r1 = iput(ncid, 0, da, T.ITYPE_SCHAR)
        e2, r2 = iput(ncid, 1, db, T.ITYPE_INT)
        err, st = N.wait_all(ncid, [r1, r2])
        exp_b, est = ora.putn(fmt, T.NC_BYTE, iv, T.ITYPE_INT, T.fill_bytes(T.NC_BYTE))
        assert st == [0, est] and est == T.NC_ERANGE
        ga = torch.zeros(n, dtype=torch.int8, device="cuda")
        gb = torch.zeros(n, dtype=torch.int32, device="cuda")
        e1, r1 = iget(ncid, 0, ga, T.ITYPE_SCHAR)
        e2, r2 = iget(ncid, 1, gb, T.ITYPE_INT)
        err, st = N.wait_all(ncid, [r1, r2])
        assert err == 0 and st == [0, 0]
        assert N.close(ncid) == 0
        raw = open(p, "rb").read()
        assert _var(raw, "a")[:n] == sc.tobytes()
        assert _var(raw, "b")[:n] == exp_b
        assert np.array_equal(ga.cpu().numpy(), sc)
        exp_i, _ = ora.getn(fmt, T.NC_BYTE, exp_b, T.ITYPE_INT)
        assert gb.cpu().numpy().tobytes() == exp_i.tobytes()


def test_bput_vara_varn_from_dev(torch_cuda, tmp_path):
    """bput_vara and bput_varn from HBM: converted into the attached buffer
    at post (NC_ERANGE at post), the user buffer reusable at once, written
    at wait"""
    torch = torch_cuda
    ora = OracleConv()
    n = 600
    rng = np.random.default_rng(5)
    f = rng.uniform(-4e4, 4e4, n).astype(np.float32)      # float -> NC_SHORT, some out of range
    p = str(tmp_path / "bp.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", n)
    N.def_var(ncid, "s", T.NC_SHORT, [0])
    N.def_var(ncid, "t", T.NC_SHORT, [0])
    assert N.enddef(ncid) == 0
    assert N.buffer_attach(ncid, 4 * n) == 0
    df = _dev(torch, f)
    e, r1 = bput(ncid, 0, df, T.ITYPE_FLOAT, start=[0], count=[n])
    assert e == T.NC_ERANGE
    df.fill_(0)                                           # the buffer is free once bput returned
    # varn: two boxes [400, 600) then [0, 400) from one device buffer
    dg = _dev(torch, f)
    ks, ps = N._ptr_array([[400], [0]])
    kc, pc = N._ptr_array([[200], [400]])
    rr = ctypes.c_int(N.NC_REQ_NULL)
    e = N.lib().pncx_nc_bput_varn(ncid, 1, 2, ps, pc, _ptr(dg), T.ITYPE_FLOAT, ctypes.byref(rr))
    assert e == T.NC_ERANGE
    dg.fill_(0)
    err, st = N.wait_all(ncid, [r1, rr.value])
    assert err == 0 and st == [0, 0]                      # NC_ERANGE was reported at post
    assert N.buffer_detach(ncid) == 0
    assert N.close(ncid) == 0
    raw = open(p, "rb").read()
    exp_s, est = ora.putn(5, T.NC_SHORT, f, T.ITYPE_FLOAT, T.fill_bytes(T.NC_SHORT))
    assert est == T.NC_ERANGE
    assert _var(raw, "s")[:2 * n] == exp_s
    # box 1 took f[0:200] into [400, 600), box 2 f[200:600] into [0, 400)
    a, _ = ora.putn(5, T.NC_SHORT, f[:200], T.ITYPE_FLOAT, T.fill_bytes(T.NC_SHORT))
    b, _ = ora.putn(5, T.NC_SHORT, f[200:], T.ITYPE_FLOAT, T.fill_bytes(T.NC_SHORT))
    assert _var(raw, "t")[:2 * n] == b + a


def test_overlapping_host_buffers_in_one_wait(torch_cuda, tmp_path):
    """Host buffers reach the batch kernels directly when every segment can
    be pinned or registered whole (zero-copy batch).  Two iput requests over
    overlapping parts of one buffer in one wait_all: the second starts inside
    the first's registration and runs past its end, so it cannot be mapped
    whole; the batch falls back to staging and converts both correctly"""
    ora = OracleConv()
    n = 1 << 18
    buf = (np.arange(n, dtype=np.int64) * 2654435761 % (1 << 31)).astype(np.int32)
    p = str(tmp_path / "ov.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    m = 3 * n // 4
    N.def_dim(ncid, "x", m)
    N.def_var(ncid, "a", T.NC_INT, [0])
    N.def_var(ncid, "b", T.NC_DOUBLE, [0])
    assert N.enddef(ncid) == 0
    va, vb = buf[:m], buf[n // 4:]                     # overlap: [n/4, 3n/4)
    e1, r1 = iput(ncid, 0, va, T.ITYPE_INT)
    e2, r2 = iput(ncid, 1, vb, T.ITYPE_INT)
    err, st = N.wait_all(ncid, [r1, r2])
    assert (e1, e2, err, st) == (0, 0, 0, [0, 0])
    assert N.close(ncid) == 0
    raw = open(p, "rb").read()
    for name, xt, vals in (("a", T.NC_INT, va), ("b", T.NC_DOUBLE, vb)):
        exp, est = ora.putn(5, xt, np.ascontiguousarray(vals), T.ITYPE_INT, T.fill_bytes(xt))
        assert est == 0 and _var(raw, name) == exp, name
