"""Reference nonblocking test programs (test/nonblocking/) restated at the
file level, one rank, CDF-1/2/5.  They exercise the aggregation at wait
time: requests whose file regions interleave, requests
waited on with NC_REQ_ALL, and put buffers that must come back unchanged.

  interleaved.c  three iput_vara into var0 whose regions interleave in file
                 order (8 x 2 columns against two 1 x 5 rows), and four into
                 var1 that tile a 3 x 10 block from pieces of one buffer
  req_all.c      iput_vara of NC_INT and NC_FLOAT variables, waited on with
                 NC_REQ_ALL
  test_bput.c    transposing bput_varm through an attached buffer, then
                 NC_ENULLABUF after detach
  wait_after_indep.c  bput_vars into a record variable, waited on later

Every cell of each variable is compared with a numpy model of the writes,
which covers the cells the reference checks and the ones it leaves out.
"""
import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N

pytestmark = pytest.mark.gpu
FORMATS = [("cdf1", 0), ("cdf2", N.NC_64BIT_OFFSET), ("cdf5", N.NC_64BIT_DATA)]


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_interleaved(gpu, tmp_path, fmt, cmode):
    ny, nx = 10, 18
    p = str(tmp_path / f"interleaved_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", ny)[1], N.def_dim(ncid, "X", nx)[1]]
    v0 = N.def_var(ncid, "var0", T.NC_INT, dims)[1]
    v1 = N.def_var(ncid, "var1", T.NC_INT, dims)[1]
    assert N.set_fill(ncid, N.NC_FILL)[0] == 0
    assert N.enddef(ncid) == 0
    model = {v0: np.full((ny, nx), -1, np.int32), v1: np.full((ny, nx), -1, np.int32)}

    def iput(v, buf, start, count):
        err, req = N.iput_var(ncid, v, buf, start=start, count=count)
        assert err == 0
        sl = tuple(slice(s, s + c) for s, c in zip(start, count))
        model[v][sl] = buf[:count[0] * count[1]].reshape(count)
        return req

    buf = np.full(ny * nx, -1, np.int32)
    assert N.put_var(ncid, v0, buf) == 0                    # var0 all -1
    buf0 = 50 + np.arange(16, dtype=np.int32)
    buf1 = 60 + np.arange(5, dtype=np.int32)
    buf2 = 70 + np.arange(5, dtype=np.int32)
    reqs = [iput(v0, buf0, [0, 3], [8, 2]), iput(v0, buf1, [1, 8], [1, 5]), iput(v0, buf2, [3, 7], [1, 5])]
    err, st = N.wait_all(ncid, reqs)
    assert err == 0 and st == [0, 0, 0]

    assert N.put_var(ncid, v1, buf) == 0                    # var1 all -1
    i = np.arange(30)
    want = np.where(i < 5, 10 + i, np.where(i < 10, 15 + i, np.where(i < 15, 20 + i,
                    np.where(i < 20, i, np.where(i < 25, 5 + i, 10 + i))))).astype(np.int32)
    buf[:30] = want
    reqs = [iput(v1, buf0, [0, 3], [8, 2]), iput(v1, buf[0:], [6, 7], [3, 5]),
            iput(v1, buf[15:], [6, 12], [2, 5]), iput(v1, buf[25:], [8, 12], [1, 5])]
    err, st = N.wait_all(ncid, reqs)
    assert err == 0 and st == [0] * 4
    assert np.array_equal(buf0, 50 + np.arange(16)) and np.array_equal(buf[:30], want)   # not altered
    assert N.close(ncid) == 0

    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    for v in (v0, v1):
        got = np.full(ny * nx, -2, np.int32)
        assert N.get_var(ncid, v, got) == 0
        assert np.array_equal(got.reshape(ny, nx), model[v]), v
    g = np.empty(ny * nx, np.int32)
    assert N.get_var(ncid, v1, g) == 0                      # the reference's own check: 10.. over 6..8 x 7..16
    assert np.array_equal(g.reshape(ny, nx)[6:9, 7:17].reshape(-1), 10 + np.arange(30))
    assert N.close(ncid) == 0


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_req_all(gpu, tmp_path, fmt, cmode):
    ny, nx, rank = 8, 2, 0
    p = str(tmp_path / f"req_all_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", ny)[1], N.def_dim(ncid, "X", nx)[1]]
    vi = N.def_var(ncid, "var_int", T.NC_INT, dims)[1]
    vf = N.def_var(ncid, "var_flt", T.NC_FLOAT, dims)[1]
    assert N.enddef(ncid) == 0
    bi = np.full(ny * nx, rank + 10, np.int32)
    bf = np.full(ny * nx, 10.5 + rank, np.float32)
    for v, b in ((vi, bi), (vf, bf)):
        assert N.iput_var(ncid, v, b, start=[0, nx * rank], count=[ny, nx])[0] == 0
    assert N.wait_all(ncid)[0] == 0                         # NC_REQ_ALL
    assert (bi == rank + 10).all() and (bf == 10.5 + rank).all()
    assert N.close(ncid) == 0
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    gi, gf = np.zeros(ny * nx, np.int32), np.zeros(ny * nx, np.float32)
    assert N.get_var(ncid, vi, gi) == 0 and N.get_var(ncid, vf, gf) == 0
    assert (gi == rank + 10).all() and (gf == np.float32(10.5 + rank)).all()
    assert N.close(ncid) == 0


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_bput(gpu, tmp_path, fmt, cmode):
    """test/nonblocking/test_bput.c: two transposing bput_varm_float into a
    6 x 4 NC_INT variable through a 4*6*sizeof(int) attached buffer; the
    float -> int conversion truncates 50.5 + k to 50 + k; a bput after
    detach is NC_ENULLABUF"""
    p = str(tmp_path / f"bput_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", 6)[1], N.def_dim(ncid, "X", 4)[1]]
    varid = N.def_var(ncid, "var", T.NC_INT, dims)[1]
    assert N.enddef(ncid) == 0
    var = (50.5 + np.arange(24)).astype(np.float32)              # var[4][6]
    keep = var.copy()
    assert N.buffer_attach(ncid, 4 * 6 * 4) == 0
    args = dict(count=[6, 2], stride=[1, 1], imap=[1, 6])
    err0, r0 = N.bput_var(ncid, varid, var, start=[0, 0], **args)
    assert err0 == 0 and np.array_equal(var, keep)
    err1, r1 = N.bput_var(ncid, varid, var[12:], start=[0, 2], **args)   # &var[2][0]
    assert err1 == 0 and np.array_equal(var, keep)
    err, st = N.wait_all(ncid, [r0, r1])
    assert err == 0 and st == [0, 0]
    assert N.buffer_detach(ncid) == 0
    assert np.array_equal(var, keep)
    assert N.bput_var(ncid, varid, var, start=[0, 0], count=[1, 1])[0] == N.NC_ENULLABUF
    assert N.close(ncid) == 0
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    got = np.empty(24, np.int32)
    assert N.get_var(ncid, varid, got) == 0
    # "ncmpidump -v var": 50, 56, 62, 68 / 51, 57, 63, 69 / ... / 55, 61, 67, 73
    assert np.array_equal(got.reshape(6, 4), (50 + np.arange(24)).reshape(4, 6).T)
    assert N.close(ncid) == 0


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_wait_after_indep(gpu, tmp_path, fmt, cmode):
    """test/nonblocking/wait_after_indep.c, one rank: a bput_vars_schar into
    a record NC_BYTE variable through an attached buffer of exactly NY*NX
    bytes, waited on later; the buffer is unchanged and the records land
    (the independent/collective mode switch has no counterpart here)"""
    ny, nx, rank = 4, 10, 0
    p = str(tmp_path / f"wait_after_indep_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", N.NC_UNLIMITED)[1], N.def_dim(ncid, "X", nx)[1]]
    varid = N.def_var(ncid, "var", T.NC_BYTE, dims)[1]
    assert N.enddef(ncid) == 0
    buf = np.full(ny * nx, rank + 10, np.int8)
    assert N.buffer_attach(ncid, ny * nx) == 0
    err, req = N.bput_var(ncid, varid, buf, start=[0, rank], count=[ny, nx], stride=[1, 1])
    assert err == 0 and (buf == rank + 10).all()
    err, st = N.wait_all(ncid, [req])
    assert err == 0 and st == [0] and (buf == rank + 10).all()
    assert N.buffer_detach(ncid) == 0
    assert N.close(ncid) == 0
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    got = np.zeros(ny * nx, np.int8)
    assert N.get_var(ncid, varid, got, start=[0, 0], count=[ny, nx]) == 0 and (got == rank + 10).all()
    assert N.close(ncid) == 0
