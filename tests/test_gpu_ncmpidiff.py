"""ncmpidiff data comparison on the GPU: the first-difference kernel against a
numpy restatement of CHECK_VAR_DIFF (ncmpidiff_core.c:200-236), and the
tool end to end on the reference's tst_file.nc."""
import io
import os
import shutil
import sys

import numpy as np
import pytest

from pnetcdf_amd import ncfile as N
from pnetcdf_amd import ncmpidiff as D
from pnetcdf_amd import nctypes as T

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TST = os.path.join(ROOT, "tests", "golden", "tst_file.nc")

TYPES = [(T.ITYPE_SCHAR, np.int8), (T.ITYPE_UCHAR, np.uint8), (T.ITYPE_SHORT, np.int16),
         (T.ITYPE_USHORT, np.uint16), (T.ITYPE_INT, np.int32), (T.ITYPE_UINT, np.uint32),
         (T.ITYPE_FLOAT, np.float32), (T.ITYPE_DOUBLE, np.float64), (T.ITYPE_LONGLONG, np.int64),
         (T.ITYPE_ULONGLONG, np.uint64)]


def ref_first_diff(a, b, tol, td, tr):
    """CHECK_VAR_DIFF, element by element semantics, vectorised: C promotion
    (int for 1/2-byte types), wrapping integer subtraction and ABS()"""
    with np.errstate(all="ignore"):
        ne = ~(a == b)
        if not tol:
            idx = np.flatnonzero(ne)
            return int(idx[0]) if idx.size else -1
        p = a.dtype
        if p.itemsize < 4 and p.kind in "iu":
            p = np.dtype(np.int32)
        pa, pb = a.astype(p), b.astype(p)
        if a.dtype.kind == "u":
            aa, ab = pa.astype(np.float64), pb.astype(np.float64)
        else:
            aa = np.where(pa >= 0, pa, -pa).astype(np.float64)
            ab = np.where(pb >= 0, pb, -pb).astype(np.float64)
        diff = np.abs((pa - pb).astype(np.float64))
        ratio = diff / np.maximum(aa, ab)
        bad = ne & ~((diff <= td) | (ratio <= tr))
        idx = np.flatnonzero(bad)
        return int(idx[0]) if idx.size else -1


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.mark.parametrize("itype,dt", TYPES)
@pytest.mark.parametrize("tol", [False, True])
@pytest.mark.parametrize("n,off", [(1, 0), (37, 1), (4099, 3), (1 << 20, 0)])
def test_first_diff_kernel(torch_cuda, itype, dt, tol, n, off):
    torch = torch_cuda
    rng = np.random.default_rng(n * 31 + itype)
    es = np.dtype(dt).itemsize
    if np.dtype(dt).kind == "f":
        a = (rng.standard_normal(n) * 100).astype(dt)
    else:
        info = np.iinfo(dt)
        a = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        a[: min(n, 2)] = [info.min, info.max][: min(n, 2)]
    b = a.copy()
    # perturbations: some within tolerance, one beyond, a NaN for floats
    k = rng.integers(0, n, size=min(n, 6))
    for j, p in enumerate(k):
        if np.dtype(dt).kind == "f":
            b[p] = a[p] * (1 + 1e-9) if j % 2 else a[p] + 5
        else:
            b[p] = a[p] ^ dt(1) if j % 2 else a[p] ^ dt(0x30)
    if np.dtype(dt).kind == "f" and n > 10:
        a[n // 2] = np.nan
        b[n // 2] = np.nan
    td, tr = 1.5, 1e-6
    exp = ref_first_diff(a, b, tol, td, tr)
    from pnetcdf_amd import ncmpidiff
    da = torch.zeros(n * es + 64, dtype=torch.uint8, device="cuda")
    db = torch.zeros(n * es + 64, dtype=torch.uint8, device="cuda")
    da[off * es:off * es + n * es] = torch.from_numpy(a.view(np.uint8).copy()).cuda()
    db[:n * es] = torch.from_numpy(b.view(np.uint8).copy()).cuda()       # different alignments
    got = ncmpidiff.first_diff(da[off * es:], db, n, itype, tol, td, tr)
    assert got == exp
    # equal arrays
    assert ncmpidiff.first_diff(da[off * es:], da[off * es:], n, itype, False, 0, 0) in (-1, n // 2 if (np.dtype(dt).kind == "f" and n > 10) else -1)


def test_first_diff_large(torch_cuda):
    torch = torch_cuda
    from pnetcdf_amd import ncmpidiff
    n = 1 << 28
    a = torch.arange(n, dtype=torch.float64, device="cuda")
    b = a.clone()
    for p in (n - 1, 123456789, 5):
        b[p] += 1
        assert ncmpidiff.first_diff(a, b, n, T.ITYPE_DOUBLE, False, 0, 0) == min(q for q in (n - 1, 123456789, 5) if b[q] != a[q])
    assert ncmpidiff.first_diff(a, b, n, T.ITYPE_DOUBLE, True, 2.0, 0) == -1


def run(*argv):
    out = io.StringIO()
    old = sys.stdout
    sys.stdout = out
    try:
        rc = D.main(list(argv))
    finally:
        sys.stdout = old
    return rc, out.getvalue().splitlines()


def test_ncmpidiff_tst_file(torch_cuda, tmp_path):
    b = str(tmp_path / "copy.nc")
    shutil.copy(TST, b)
    rc, lines = run(TST, b)
    assert rc == 0
    assert lines == ["Headers of two files are the same", "All variables of two files are the same"]
    # change one element of fix_var(Y=4, X=12) and one of rec_var(time, X)
    err, ncid = N.open(b, N.NC_WRITE)
    v = np.zeros(1, np.float32)
    assert N.get_var(ncid, 1, v, start=[2, 5], count=[1, 1]) == 0
    old = float(v[0])
    assert N.put_var(ncid, 1, np.array([old + 0.5], np.float32), start=[2, 5], count=[1, 1]) == 0
    assert N.put_var(ncid, 0, np.array([7.25], np.float32), start=[1, 11], count=[1, 1]) == 0
    assert N.close(ncid) == 0
    err, ncid = N.open(TST)
    r = np.zeros(1, np.float32)
    assert N.get_var(ncid, 0, r, start=[1, 11], count=[1, 1]) == 0
    N.close(ncid)
    rc, lines = run(TST, b)
    assert rc == 1
    new = float(np.float32(old + 0.5))
    assert lines == [
        "ncmpidiff %s %s" % (TST, b),
        'DIFF: variable "rec_var" of type "NC_FLOAT" at element [1, 11] of value %g vs %g (difference = %e)'
        % (float(r[0]), 7.25, float(r[0]) - 7.25),
        'DIFF: variable "fix_var" of type "NC_FLOAT" at element [2, 5] of value %g vs %g (difference = %e)'
        % (old, new, old - new),
        "Headers of two files are the same",
        "Number of differences in variables 2"]
    # -v selects one variable; a tolerance of 1.0 absorbs the 0.5 change
    rc, lines = run("-v", "fix_var", "-t", "1.0,0", TST, b)
    assert rc == 0 and lines == ["Compared variable(s) are the same"]
    rc, lines = run("-q", "-v", "fix_var", TST, b)
    assert rc == 1 and lines[-1].startswith('DIFF: variable "fix_var"')


def test_ncmpidiff_numeric_attributes_and_byte_quirk(torch_cuda, tmp_path):
    """numeric attribute contents (CHECK_VAR_ATT_DIFF) and the reference's
    missing NC_BYTE case: byte data and byte attributes are not compared"""
    paths = []
    for k, (scale, bval) in enumerate(((1.0, 3), (2.0, 4))):
        p = str(tmp_path / f"f{k}.nc")
        err, ncid = N.create(p, N.NC_64BIT_DATA)
        d = N.def_dim(ncid, "x", 5)[1]
        N.def_var(ncid, "v", T.NC_DOUBLE, [d])
        N.def_var(ncid, "b", T.NC_BYTE, [d])
        N.put_att(ncid, 0, "scale", T.NC_DOUBLE, np.array([scale, 0.5]))
        N.put_att(ncid, 1, "bb", T.NC_BYTE, np.array([bval], np.int8))
        assert N.enddef(ncid) == 0
        assert N.put_var(ncid, 0, np.arange(5, dtype=np.float64)) == 0
        assert N.put_var(ncid, 1, np.arange(5, dtype=np.int8) * (k + 1)) == 0
        assert N.close(ncid) == 0
        paths.append(p)
    rc, lines = run(*paths)
    assert rc == 1
    assert lines == ["ncmpidiff %s %s" % tuple(paths),
                     'DIFF: variable "v" attribute "scale" of type "NC_DOUBLE" at element 0 of value 1 vs 2 '
                     '(difference = -1.000000e+00)',
                     "Number of differences in header 1",
                     "All variables of two files are the same"]
