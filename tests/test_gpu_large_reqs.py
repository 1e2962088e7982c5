"""test/largefile/large_reqs.c restated for one rank (1 x 1 process grid):
single requests and buffers beyond 4 GiB through the file layer.

  tst_one_var: a 1280 x 1048576 NC_INT record variable (5 GiB per record):
    put/get of the whole record, of a (1152 x 1048448) part with a contiguous
    user buffer, and of that part through a subarray buftype of the full
    1280 x 1048576 buffer (MPI_Type_create_subarray, C order).
  tst_vars: 1100 record variables of 1024 x 1024 NC_INT (4.4 GiB per
    record), each written by iput_vara with a (1022 x 1022) subarray buftype
    and read by iget_vara, both completed by one wait_all.

The reference checks only the return codes; here every byte read back is
compared with what was written, and the buffer bytes outside the subarray
must survive the read.  Files go to /dev/shm when it has room (the test
needs ~6 GiB there), else to pytest's tmp_path.
"""
import os
import shutil

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N
from pnetcdf_amd import pncx

pytestmark = pytest.mark.gpu

NY, NX = 1280, 1048576
NVARS, LEN, GAP = 1100, 1024, 2


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


@pytest.fixture
def bigdir(tmp_path):
    for d in ("/dev/shm", str(tmp_path)):
        if os.path.isdir(d) and shutil.disk_usage(d).free > (7 << 30):
            path = os.path.join(d, f"pncx_large_reqs_{os.getpid()}")
            os.makedirs(path, exist_ok=True)
            yield path
            shutil.rmtree(path, ignore_errors=True)
            return
    pytest.skip("no file system with 7 GiB free")


def subarray(isz, gsize, lsize):
    """flattened MPI_Type_create_subarray(2, gsize, lsize, {0,0}, C order)"""
    disp = (np.arange(lsize[0], dtype=np.int64) * gsize[1] * isz).tolist()
    return pncx.DType(T.ITYPE_INT, disp, [lsize[1]] * lsize[0], gsize[0] * gsize[1] * isz)


def test_tst_one_var(gpu, bigdir):
    p = os.path.join(bigdir, "one_var.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | N.NC_64BIT_DATA)
    assert err == 0
    dims = [N.def_dim(ncid, "time", N.NC_UNLIMITED)[1], N.def_dim(ncid, "Y", NY)[1], N.def_dim(ncid, "X", NX)[1]]
    err, varid = N.def_var(ncid, "var", T.NC_INT, dims)
    assert err == 0 and N.enddef(ncid) == 0
    buf = np.arange(NY * NX, dtype=np.int32) & 127                             # (i + rank) % 128
    # the entire variable: one 5 GiB request each way
    assert N.put_var(ncid, varid, buf, start=[0, 0, 0], count=[1, NY, NX]) == 0
    back = np.full(NY * NX, -1, np.int32)
    assert N.get_var(ncid, varid, back, start=[0, 0, 0], count=[1, NY, NX]) == 0
    assert np.array_equal(back, buf)
    # part of it, contiguous user buffer
    cy, cx = NY - 128, NX - 128
    assert N.put_var(ncid, varid, buf[:cy * cx], start=[0, 0, 0], count=[1, cy, cx]) == 0
    back[:] = -1
    assert N.get_var(ncid, varid, back[:cy * cx], start=[0, 0, 0], count=[1, cy, cx]) == 0
    assert np.array_equal(back[:cy * cx], buf[:cy * cx]) and (back[cy * cx:] == -1).all()
    # the same part through a subarray buftype over the full NY x NX buffer
    dt = subarray(4, (NY, NX), (cy, cx))
    src = np.arange(NY * NX, dtype=np.int32) % 127                             # differs from what is on disk
    assert N.put_var_flex(ncid, varid, src, 1, dt, start=[0, 0, 0], count=[1, cy, cx]) == 0
    back[:] = -7
    assert N.get_var_flex(ncid, varid, back, 1, dt, start=[0, 0, 0], count=[1, cy, cx]) == 0
    b2, s2 = back.reshape(NY, NX), src.reshape(NY, NX)
    assert np.array_equal(b2[:cy, :cx], s2[:cy, :cx])
    assert (b2[:cy, cx:] == -7).all() and (b2[cy:, :] == -7).all()
    assert N.close(ncid) == 0
    # what the subarray put left on disk, through a plain contiguous get
    err, ncid = N.open(p)
    assert err == 0
    part = np.empty(cy * cx, np.int32)
    assert N.get_var(ncid, varid, part, start=[0, 0, 0], count=[1, cy, cx]) == 0
    assert np.array_equal(part.reshape(cy, cx), s2[:cy, :cx])
    assert N.close(ncid) == 0
    dt.free()


def test_tst_vars(gpu, bigdir):
    p = os.path.join(bigdir, "vars.nc")
    err, ncid = N.create(p, N.NC_CLOBBER | N.NC_64BIT_DATA)
    assert err == 0
    dims = [N.def_dim(ncid, "time", N.NC_UNLIMITED)[1], N.def_dim(ncid, "Y", LEN)[1], N.def_dim(ncid, "X", LEN)[1]]
    varids = []
    for i in range(NVARS):
        err, v = N.def_var(ncid, f"var.{i}", T.NC_INT, dims)
        assert err == 0
        varids.append(v)
    assert N.enddef(ncid) == 0
    n = (LEN * LEN + GAP) * NVARS
    buf = np.arange(n, dtype=np.int32) & 127
    ly = lx = LEN - GAP
    dt = subarray(4, (LEN, LEN), (ly, lx))
    reqs = []
    for i, v in enumerate(varids):                     # buf_ptr += LEN*LEN + gap
        err, r = N.iput_var_flex(ncid, v, buf, 1, dt, start=[0, 0, 0], count=[1, ly, lx],
                                 base=4 * i * (LEN * LEN + GAP))
        assert err == 0
        reqs.append(r)
    err, st = N.wait_all(ncid, reqs)
    assert err == 0 and st == [0] * NVARS
    back = np.full(n, -3, np.int32)
    reqs = []
    for i, v in enumerate(varids):                     # buf_ptr += LEN*LEN
        err, r = N.iget_var_flex(ncid, v, back, 1, dt, start=[0, 0, 0], count=[1, ly, lx], base=4 * i * LEN * LEN)
        assert err == 0
        reqs.append(r)
    err, st = N.wait_all(ncid, reqs)
    assert err == 0 and st == [0] * NVARS
    for i in range(NVARS):
        got = back[i * LEN * LEN:(i + 1) * LEN * LEN].reshape(LEN, LEN)
        want = buf[i * (LEN * LEN + GAP):i * (LEN * LEN + GAP) + LEN * LEN].reshape(LEN, LEN)
        assert np.array_equal(got[:ly, :lx], want[:ly, :lx]), i
        assert (got[:ly, lx:] == -3).all() and (got[ly:, :] == -3).all(), i
    assert (back[NVARS * LEN * LEN:] == -3).all()
    assert N.close(ncid) == 0
    dt.free()
