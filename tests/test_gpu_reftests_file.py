"""Reference test programs restated at the file level, one rank, for the
classic formats the reference loops over (CDF-1, CDF-2, CDF-5):

  test/testcases/test_varm.c   transposed varm reads (iget/get, stride NULL
                               and not) and transposed schar varm writes
                               (iput/put); the write buffer must not change
  test/testcases/flexible.c    flexible puts through hindexed buftypes with
                               a negative displacement (row swap), with and
                               without conversion (NC_INT, NC_DOUBLE, NC_BYTE),
                               fill_var_rec, and gets through a subarray
                               buftype with ghost cells (blocking and iget)
  test/testcases/vectors.c     vector(4,3,5) resized to 20 ints, 25 copies,
                               int -> NC_DOUBLE put_vara and back
  test/testcases/flexible_varm.c  a transposing imap combined with a
                               subarray buftype with ghost cells
  test/testcases/tst_vars_fill.m4  strided puts of every type with fill
                               mode on: the gaps read back as the fill value
  test/testcases/test_fillvalue.c  _FillValue type rules, a scalar variable
                               filled with its _FillValue
  test/testcases/tst_def_var_fill.c  per-variable fill mode, NC_EGLOBAL
  test/testcases/scalar.c      every put/get form on a scalar variable
  test/testcases/flexible2.c   subarray buftypes with ghost cells and type
                               conversion, blocking and nonblocking
  test/testcases/flexible_var.c  whole-variable flexible put/get/iput/iget

The MPI datatypes are given as their flattened typemaps (pncx.DType); the
MPI flattening itself is checked against MPI_Pack in tests/mpi/flex_check.c.
Expected values are the ones the reference programs assert (and, where they
only check return codes, the values their comments print).
"""
import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N
from pnetcdf_amd import pncx

pytestmark = pytest.mark.gpu
FORMATS = [("cdf1", 0), ("cdf2", N.NC_64BIT_OFFSET), ("cdf5", N.NC_64BIT_DATA)]


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_varm(gpu, tmp_path, fmt, cmode):
    p = str(tmp_path / f"varm_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", 6)[1], N.def_dim(ncid, "X", 4)[1]]
    err, varid = N.def_var(ncid, "var", T.NC_INT, dims)
    assert err == 0 and N.enddef(ncid) == 0
    var = np.arange(24, dtype=np.int32)                      # var[j][i] = j*4+i
    assert N.put_var(ncid, varid, var, start=[0, 0], count=[6, 4]) == 0
    assert N.sync(ncid) == 0 and N.close(ncid) == 0

    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    err, varid = N.inq_varid(ncid, "var")
    # rh is 4 x 6: rh[j][i] = var[i][j]  (check_read_contents)
    expect = np.arange(24, dtype=np.float32).reshape(6, 4).T.copy()
    rh = np.full((4, 6), -1.0, np.float32)
    err, req = N.iget_var(ncid, varid, rh, start=[0, 0], count=[6, 4], imap=[1, 6])
    assert err == 0
    err, st = N.wait_all(ncid, [req])
    assert err == 0 and st == [0] and np.array_equal(rh, expect)
    for stride in ([1, 1], None):
        rh[:] = -1.0
        assert N.get_var(ncid, varid, rh, start=[0, 0], count=[6, 4], stride=stride, imap=[1, 6]) == 0
        assert np.array_equal(rh, expect)
    assert N.close(ncid) == 0

    err, ncid = N.open(p, N.NC_WRITE)
    assert err == 0
    assert N.put_var(ncid, varid, np.zeros(24, np.int32), start=[0, 0], count=[6, 4]) == 0
    varT = (np.arange(24).reshape(4, 6) + 50).astype(np.int8)   # varT[j][i] = j*6+i+50
    keep = varT.copy()
    for stride in ([1, 1], None):                               # nonblocking
        err, req = N.iput_var(ncid, varid, varT, start=[0, 0], count=[6, 4], stride=stride, imap=[1, 6])
        assert err == 0
        err, st = N.wait_all(ncid, [req])
        assert err == 0 and st == [0] and np.array_equal(varT, keep)   # check_write_contents
    for stride in ([1, 1], None):                               # blocking
        assert N.put_var(ncid, varid, varT, start=[0, 0], count=[6, 4], stride=stride, imap=[1, 6]) == 0
        assert np.array_equal(varT, keep)
    # "ncmpidump -v var": 50, 56, 62, 68 / 51, 57, 63, 69 / ...
    got = np.empty(24, np.int32)
    assert N.get_var(ncid, varid, got, start=[0, 0], count=[6, 4]) == 0
    assert np.array_equal(got.reshape(6, 4), keep.T.astype(np.int32))
    assert N.close(ncid) == 0


NY, NX = 2, 70


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_flexible(gpu, tmp_path, fmt, cmode):
    p = str(tmp_path / f"flexible_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", N.NC_UNLIMITED)[1], N.def_dim(ncid, "X", NX)[1]]
    v1 = N.def_var(ncid, "var_int", T.NC_INT, dims)[1]
    v2 = N.def_var(ncid, "var_dbl", T.NC_DOUBLE, dims)[1]
    v3 = N.def_var(ncid, "var_byte", T.NC_BYTE, dims)[1]
    assert N.set_fill(ncid, N.NC_FILL)[0] == 0
    assert N.enddef(ncid) == 0
    for v in (v1, v2, v3):
        for rec in (0, 1):
            assert N.fill_var_rec(ncid, v, rec) == 0
    buf = np.empty((NY, NX), np.int32)
    for j in range(NY):
        buf[j, :] = j + 10                                   # j + rank + 10
    keep = buf.copy()
    # hindexed(2, {NX, NX}, {0, buf[0]-buf[1]}, MPI_INT) applied at bufptr = buf[1]: row 1 then row 0
    swap = pncx.DType(T.ITYPE_INT, [0, -NX * 4], [NX, NX], 2 * NX * 4)
    for v in (v1, v2):                                       # no conversion, then int -> double
        assert N.put_var_flex(ncid, v, buf, 1, swap, start=[0, 0], count=[2, NX], base=NX * 4) == 0
        assert np.array_equal(buf, keep)
    schar = np.empty(NY * NX, np.int8)
    for j in range(NY):
        schar[j * NX:(j + 1) * NX] = j + 10
    keep_c = schar.copy()
    swap_c = pncx.DType(T.ITYPE_SCHAR, [0, -NX], [NX, NX], 2 * NX)
    assert N.put_var_flex(ncid, v3, schar, 1, swap_c, start=[0, 0], count=[2, NX], base=NX) == 0
    assert np.array_equal(schar, keep_c)
    schar[:] = -1
    assert N.get_var_flex(ncid, v3, schar, 1, swap_c, start=[0, 0], count=[2, NX], base=NX) == 0
    assert np.array_equal(schar, keep_c)
    assert N.sync(ncid) == 0 and N.close(ncid) == 0

    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    expect = np.empty((NY, NX), np.int32)
    expect[0, :], expect[1, :] = 11, 10                      # rows swapped by the buftype
    for v in (v1, v2):
        buf[:] = -1
        assert N.get_var(ncid, v, buf, start=[0, 0], count=[2, NX]) == 0
        assert np.array_equal(buf, expect)
    # subarray buftype with 2 ghost cells on each side
    gy, gx = NY + 4, NX + 4
    ghost = pncx.DType(T.ITYPE_INT, [((r + 2) * gx + 2) * 4 for r in range(NY)], [NX] * NY, gy * gx * 4)
    nc = np.full(gy * gx, -1, np.int32)
    for v in (v1, v2):
        for nonblocking in (False, True):
            nc[:] = -1
            if nonblocking:
                err, req = N.iget_var_flex(ncid, v, nc, 1, ghost, start=[0, 0], count=[2, NX])
                assert err == 0
                err, st = N.wait_all(ncid, [req])
                assert err == 0 and st == [0]
            else:
                assert N.get_var_flex(ncid, v, nc, 1, ghost, start=[0, 0], count=[2, NX]) == 0
            g = nc.reshape(gy, gx)
            assert np.array_equal(g[2:2 + NY, 2:2 + NX], expect)
            inner = np.zeros((gy, gx), bool)
            inner[2:2 + NY, 2:2 + NX] = True
            assert (g[~inner] == -1).all()
    assert N.close(ncid) == 0
    for d in (swap, swap_c, ghost):
        d.free()


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_vectors(gpu, tmp_path, fmt, cmode):
    VECCOUNT, BLOCKLEN, STRIDE, COUNT = 4, 3, 5, 25
    p = str(tmp_path / f"vectors_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    err, dimid = N.def_dim(ncid, "50k", 1024 * 50)
    err, varid = N.def_var(ncid, "vector", T.NC_DOUBLE, [dimid])
    assert N.def_var_fill(ncid, varid, 0, None) == 0
    assert N.enddef(ncid) == 0
    # MPI_Type_vector(4, 3, 5, MPI_INT) resized to 20 ints, 25 copies
    vec = pncx.DType(T.ITYPE_INT, [b * STRIDE * 4 for b in range(VECCOUNT)], [BLOCKLEN] * VECCOUNT,
                     STRIDE * VECCOUNT * 4)
    nuser = STRIDE * VECCOUNT * COUNT
    userbuf = (3.14159 * np.arange(nuser)).astype(np.int32)      # userbuf[i] = pi*i
    start, acount = 10, COUNT * 12
    assert N.put_var_flex(ncid, varid, userbuf, COUNT, vec, start=[start], count=[acount]) == 0
    assert N.sync(ncid) == 0 and N.close(ncid) == 0
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    cmpbuf = np.zeros(nuser, np.int32)
    assert N.get_var_flex(ncid, varid, cmpbuf, COUNT, vec, start=[start], count=[acount]) == 0
    # the reference compares i < acount with i % STRIDE < BLOCKLEN; every
    # typemap element is compared here, and the gaps must stay zero
    sel = (np.arange(nuser) % STRIDE) < BLOCKLEN
    assert np.array_equal(cmpbuf[sel], userbuf[sel]) and not cmpbuf[~sel].any()
    # on disk: the packed elements as doubles, fill value around them
    got = np.empty(1024 * 50, np.float64)
    assert N.get_var(ncid, varid, got) == 0
    assert np.array_equal(got[start:start + acount], userbuf[sel].astype(np.float64))
    assert (got[:start] == T.XTYPE_FILL[T.NC_DOUBLE]).all()
    assert (got[start + acount:] == T.XTYPE_FILL[T.NC_DOUBLE]).all()
    assert N.close(ncid) == 0
    vec.free()


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_flexible_varm(gpu, tmp_path, fmt, cmode):
    """test/testcases/flexible_varm.c: a transposing imap ({1, NY} on count
    {NY, NX}) combined with a subarray buftype of an (NX+4) x (NY+4) int
    buffer with 2 ghost cells, NC_DOUBLE variable; put/iput leave the buffer
    unchanged, get/iget fill the interior and leave the ghosts"""
    ny, nx, gh = 32, 128, 2
    gx, gy = nx + 2 * gh, ny + 2 * gh                     # buf[NX+2G][NY+2G]
    sub = pncx.DType(T.ITYPE_INT, [((r + gh) * gy + gh) * 4 for r in range(nx)], [ny] * nx, gx * gy * 4)
    inner = np.zeros((gx, gy), bool)
    inner[gh:gh + nx, gh:gh + ny] = True
    put = np.full((gx, gy), -1, np.int32)                 # INIT_PUT_BUF
    put[gh:gh + nx, gh:gh + ny] = np.arange(nx * ny, dtype=np.int32).reshape(nx, ny)
    keep = put.copy()
    p = str(tmp_path / f"flexible_varm_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", ny)[1], N.def_dim(ncid, "X", nx)[1]]
    err, varid = N.def_var(ncid, "var", T.NC_DOUBLE, dims)
    assert err == 0 and N.enddef(ncid) == 0
    args = dict(start=[0, 0], count=[ny, nx], stride=[1, 1], imap=[1, ny])
    assert N.put_var_flex(ncid, varid, put, 1, sub, **args) == 0
    assert np.array_equal(put, keep)                      # CHECK_PUT_BUF
    err, req = N.iput_var_flex(ncid, varid, put, 1, sub, **args)
    assert err == 0
    err, st = N.wait_all(ncid, [req])
    assert err == 0 and st == [0] and np.array_equal(put, keep)
    assert N.sync(ncid) == 0
    # on disk: var[y][x] = packed element x*NY + y (the transposing imap)
    disk = np.empty(ny * nx, np.float64)
    assert N.get_var(ncid, varid, disk) == 0
    assert np.array_equal(disk.reshape(ny, nx), np.arange(nx * ny, dtype=np.float64).reshape(nx, ny).T)
    for nonblocking in (False, True):
        got = np.full((gx, gy), -2, np.int32)             # INIT_GET_BUF
        if nonblocking:
            err, req = N.iget_var_flex(ncid, varid, got, 1, sub, **args)
            assert err == 0
            err, st = N.wait_all(ncid, [req])
            assert err == 0 and st == [0]
        else:
            assert N.get_var_flex(ncid, varid, got, 1, sub, **args) == 0
        assert np.array_equal(got[inner], keep[inner]) and (got[~inner] == -2).all()   # CHECK_GET_BUF
    assert N.close(ncid) == 0
    sub.free()


# NC_TYPE(itype) of the m4 test: schar->NC_BYTE, uchar->NC_UBYTE, ..., the unsigned and 64-bit ones CDF-5 only
VARS_FILL_TYPES = [(np.int8, T.NC_BYTE, False), (np.uint8, T.NC_UBYTE, True), (np.int16, T.NC_SHORT, False),
                   (np.uint16, T.NC_USHORT, True), (np.int32, T.NC_INT, False), (np.uint32, T.NC_UINT, True),
                   (np.float32, T.NC_FLOAT, False), (np.float64, T.NC_DOUBLE, False),
                   (np.int64, T.NC_INT64, True), (np.uint64, T.NC_UINT64, True)]


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_tst_vars_fill(gpu, tmp_path, fmt, cmode):
    """test/testcases/tst_vars_fill.m4: fill mode on, put_vars with strides
    2..5 in both dimensions into 16 x 16 variables of every type, get_vara of
    the whole variable: written points hold the value, every other point the
    type's default fill value (NC_FILL_VALUE(itype))"""
    NYF = NXF = 16
    for dt, xt, cdf5_only in VARS_FILL_TYPES:
        if cdf5_only and cmode != N.NC_64BIT_DATA:
            continue
        p = str(tmp_path / f"vars_fill_{fmt}_{np.dtype(dt).name}.nc")
        err, ncid = N.create(p, N.NC_CLOBBER | cmode)
        assert err == 0
        dims = [N.def_dim(ncid, "Y", NYF)[1], N.def_dim(ncid, "X", NXF)[1]]
        assert N.set_fill(ncid, N.NC_FILL)[0] == 0
        varids = [N.def_var(ncid, f"var_{k}", xt, dims)[1] for k in range(4)]
        assert N.enddef(ncid) == 0
        for k, v in enumerate(varids):
            s = 2 + k
            cnt = [-(-NYF // s), -(-NXF // s)]                  # count++ when NY % stride
            buf = np.zeros(NYF * NXF, dt)                        # ($1)rank
            assert N.put_var(ncid, v, buf[:cnt[0] * cnt[1]], start=[0, 0], count=cnt, stride=[s, s]) == 0
            assert N.sync(ncid) == 0
            got = np.ones(NYF * NXF, dt)
            assert N.get_var(ncid, v, got, start=[0, 0], count=[NYF, NXF]) == 0
            g = got.reshape(NYF, NXF)
            written = np.zeros((NYF, NXF), bool)
            written[::s, ::s] = True
            assert (g[written] == 0).all(), (np.dtype(dt).name, k)
            assert (g[~written] == dt(T.XTYPE_FILL[xt])).all(), (np.dtype(dt).name, k)
        assert N.close(ncid) == 0


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_fillvalue(gpu, tmp_path, fmt, cmode):
    """test/testcases/test_fillvalue.c: a global _FillValue of any type is
    allowed; a variable's must have the variable's type (NC_EBADTYPE); the
    scalar NC_INT variable, never written, reads back its _FillValue 5678"""
    p = str(tmp_path / f"fillvalue_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    assert N.put_att(ncid, N.NC_GLOBAL, "_FillValue", T.NC_FLOAT, np.array([1.234], np.float32)) == 0
    err, varid = N.def_var(ncid, "var", T.NC_INT, [])
    assert err == 0
    assert N.put_att(ncid, varid, "_FillValue", T.NC_FLOAT, np.array([1.234], np.float32)) == N.NC_EBADTYPE
    assert N.put_att(ncid, varid, "_FillValue", T.NC_INT, np.array([5678], np.int32)) == 0
    assert N.set_fill(ncid, N.NC_FILL)[0] == 0
    assert N.close(ncid) == 0                               # enddef through close
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    got = np.zeros(1, np.int32)
    assert N.get_var(ncid, varid, got) == 0 and got[0] == 5678
    assert N.close(ncid) == 0


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_tst_def_var_fill(gpu, tmp_path, fmt, cmode):
    """test/testcases/tst_def_var_fill.c, one rank: def_var_fill on NC_GLOBAL
    is NC_EGLOBAL; var_nofill and var_fill get columns 2..3 of an NY x NX
    NC_INT variable; var_fill reads NC_FILL_INT everywhere else"""
    ny, nx, rank = 8, 5, 0
    p = str(tmp_path / f"def_var_fill_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", ny)[1], N.def_dim(ncid, "X", nx)[1]]
    v0 = N.def_var(ncid, "var_nofill", T.NC_INT, dims)[1]
    v1 = N.def_var(ncid, "var_fill", T.NC_INT, dims)[1]
    assert N.def_var_fill(ncid, N.NC_GLOBAL, 1, None) == N.NC_EGLOBAL
    assert N.def_var_fill(ncid, v0, 1, None) == 0
    assert N.def_var_fill(ncid, v1, 0, None) == 0
    assert N.enddef(ncid) == 0
    assert N.fill_var_rec(ncid, N.NC_GLOBAL, 0) == N.NC_EGLOBAL
    buf = np.full(ny * nx, rank + 5, np.int32)
    for v in (v0, v1):
        assert N.put_var(ncid, v, buf[:ny * 2], start=[0, nx * rank + 2], count=[ny, 2]) == 0
        assert (buf == rank + 5).all()                      # put buffer not altered
    assert N.sync(ncid) == 0 and N.close(ncid) == 0
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    assert N.inq_var_fill(ncid, N.NC_GLOBAL, np.int32)[0] == N.NC_EGLOBAL
    cols = np.zeros((ny, nx), bool)
    cols[:, 2:4] = True
    for v, filled in ((v0, False), (v1, True)):
        got = np.full(ny * nx, -1, np.int32)
        assert N.get_var(ncid, v, got, start=[0, 0], count=[ny, nx]) == 0
        g = got.reshape(ny, nx)
        assert (g[cols] == rank + 5).all()
        if filled:
            assert (g[~cols] == T.XTYPE_FILL[T.NC_INT]).all()
    assert N.close(ncid) == 0


SCALAR_ARGS = [dict(start=None), dict(start=[1]), dict(start=[1], count=[2]), dict(count=[2]),
               dict(start=[1], count=None), dict(), dict(start=[1], count=[2], stride=[2]),
               dict(count=[2], stride=[2]), dict(start=[1], stride=[2]), dict(start=[1], count=[2]),
               dict(start=[1], count=[2], stride=[2], imap=[2])]


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_scalar(gpu, tmp_path, fmt, cmode):
    """test/testcases/scalar.c: on a scalar variable every put/get form
    (var1/vara/vars/varm, blocking and nonblocking) succeeds and ignores
    start, count, stride and imap, NULL or not"""
    p = str(tmp_path / f"scalar_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    err, varid = N.def_var(ncid, "scalar_var", T.NC_INT, [])
    assert err == 0 and N.enddef(ncid) == 0
    for k, a in enumerate(SCALAR_ARGS):
        buf = np.array([k + 1], np.int32)
        assert N.put_var(ncid, varid, buf, **a) == 0, a
        err, req = N.iput_var(ncid, varid, buf, **a)
        assert err == 0, a
        assert N.wait_all(ncid)[0] == 0
    assert N.sync(ncid) == 0 and N.close(ncid) == 0
    err, ncid = N.open(p, N.NC_NOWRITE)
    assert err == 0
    err, varid = N.inq_varid(ncid, "scalar_var")
    for a in SCALAR_ARGS:
        got = np.zeros(1, np.int32)
        assert N.get_var(ncid, varid, got, **a) == 0 and got[0] == len(SCALAR_ARGS), a
        got[0] = 0
        err, req = N.iget_var(ncid, varid, got, **a)
        assert err == 0, a
        assert N.wait_all(ncid)[0] == 0 and got[0] == len(SCALAR_ARGS), a
    assert N.close(ncid) == 0


def subarray(itype, esize, sizes, subsizes, starts):
    """MPI_Type_create_subarray(2, ..., MPI_ORDER_C) as its flattened typemap"""
    disp = [((r + starts[0]) * sizes[1] + starts[1]) * esize for r in range(subsizes[0])]
    return pncx.DType(itype, disp, [subsizes[1]] * subsizes[0], sizes[0] * sizes[1] * esize)


def ghost_mask(sizes, subsizes, g):
    m = np.zeros(sizes, bool)
    m[g:g + subsizes[0], g:g + subsizes[1]] = True
    return m


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_flexible2(gpu, tmp_path, fmt, cmode):
    """test/testcases/flexible2.c, one rank: subarray buftypes with 3 ghost
    cells and type conversion -- int buffer into NC_INT var_zy (blocking
    put/get), double buffer into NC_FLOAT var_yx (iput/iget + wait)"""
    nz, ny, nx, g, rank = 5, 5, 70, 3, 0
    p = str(tmp_path / f"flexible2_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dz, dy, dx = N.def_dim(ncid, "Z", nz)[1], N.def_dim(ncid, "Y", ny)[1], N.def_dim(ncid, "X", nx)[1]
    v0 = N.def_var(ncid, "var_zy", T.NC_INT, [dz, dy])[1]
    v1 = N.def_var(ncid, "var_yx", T.NC_FLOAT, [dy, dx])[1]
    assert N.enddef(ncid) == 0

    sizes, sub = (nz + 2 * g, ny + 2 * g), (nz, ny)
    st = subarray(T.ITYPE_INT, 4, sizes, sub, (g, g))
    buf = np.full(sizes, rank + 10, np.int32)
    args = dict(start=[nz * rank, 0], count=[nz, ny])
    assert N.put_var_flex(ncid, v0, buf, 1, st, **args) == 0
    assert (buf == rank + 10).all()
    assert N.sync(ncid) == 0
    buf[:] = -1
    assert N.get_var_flex(ncid, v0, buf, 1, st, **args) == 0
    m = ghost_mask(sizes, sub, g)
    assert (buf[m] == rank + 10).all() and (buf[~m] == -1).all()
    st.free()

    sizes, sub = (ny + 2 * g, nx + 2 * g), (ny, nx)
    st = subarray(T.ITYPE_DOUBLE, 8, sizes, sub, (g, g))
    buf = np.full(sizes, rank + 10, np.float64)
    args = dict(start=[0, nx * rank], count=[ny, nx])
    err, req = N.iput_var_flex(ncid, v1, buf, 1, st, **args)
    assert err == 0
    err, s = N.wait_all(ncid, [req])
    assert err == 0 and s == [0] and (buf == rank + 10).all()
    buf[:] = -1
    err, req = N.iget_var_flex(ncid, v1, buf, 1, st, **args)
    assert err == 0
    err, s = N.wait_all(ncid, [req])
    m = ghost_mask(sizes, sub, g)
    assert err == 0 and s == [0] and (buf[m] == rank + 10).all() and (buf[~m] == -1).all()
    st.free()
    assert N.close(ncid) == 0


@pytest.mark.parametrize("fmt,cmode", FORMATS)
def test_flexible_var(gpu, tmp_path, fmt, cmode):
    """test/testcases/flexible_var.c, one rank: put_var/get_var/iput_var/
    iget_var of a whole NY x NX NC_DOUBLE variable through a subarray int
    buftype with 2 ghost cells (bufcount 1), then with a plain int buffer
    (the reference's bufcount = NC_COUNT_IGNORE with MPI_INT)"""
    ny, nx, g = 32, 128, 2
    p = str(tmp_path / f"flexible_var_{fmt}.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | cmode)
    assert err == 0
    dims = [N.def_dim(ncid, "Y", ny)[1], N.def_dim(ncid, "X", nx)[1]]
    varid = N.def_var(ncid, "var", T.NC_DOUBLE, dims)[1]
    assert N.enddef(ncid) == 0
    sizes, sub = (ny + 2 * g, nx + 2 * g), (ny, nx)
    st = subarray(T.ITYPE_INT, 4, sizes, sub, (g, g))
    m = ghost_mask(sizes, sub, g)
    inner = np.arange(ny * nx, dtype=np.int32)

    def put_buf():                                          # INIT_PUT_BUF_GHOST
        b = np.full(sizes, -1, np.int32)
        b[m] = inner
        return b

    def check_get(b):                                       # CHECK_GET_BUF_GHOST
        assert np.array_equal(b[m], inner) and (b[~m] == -2).all()

    def get_both():
        b = np.full(sizes, -2, np.int32)                    # INIT_GET_BUF
        assert N.get_var_flex(ncid, varid, b, 1, st) == 0
        check_get(b)
        b[:] = -2
        err, req = N.iget_var_flex(ncid, varid, b, 1, st)
        assert err == 0 and N.wait_all(ncid, [req]) == (0, [0])
        check_get(b)

    b = put_buf()
    assert N.put_var_flex(ncid, varid, b, 1, st) == 0
    assert np.array_equal(b, put_buf())                     # CHECK_PUT_BUF_GHOST
    get_both()
    assert N.put_var(ncid, varid, np.zeros(ny * nx, np.int32)) == 0
    b = put_buf()
    err, req = N.iput_var_flex(ncid, varid, b, 1, st)
    assert err == 0 and np.array_equal(b, put_buf())
    assert N.wait_all(ncid, [req]) == (0, [0])
    get_both()
    st.free()

    plain = inner.copy()                                    # no ghost cells
    assert N.put_var(ncid, varid, plain) == 0 and np.array_equal(plain, inner)
    for nonblocking in (False, True):
        got = np.full(ny * nx, -2, np.int32)
        if nonblocking:
            err, req = N.iget_var(ncid, varid, got)
            assert err == 0 and N.wait_all(ncid, [req]) == (0, [0])
        else:
            assert N.get_var(ncid, varid, got) == 0
        assert np.array_equal(got, inner)
    err, req = N.iput_var(ncid, varid, plain)
    assert err == 0 and N.wait_all(ncid, [req]) == (0, [0]) and np.array_equal(plain, inner)
    disk = np.empty(ny * nx, np.float64)
    assert N.get_var(ncid, varid, disk) == 0 and np.array_equal(disk, inner.astype(np.float64))
    assert N.close(ncid) == 0
