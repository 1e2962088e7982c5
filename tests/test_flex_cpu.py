"""Flexible API host logic (CPU, no GPU): MPI datatype flattening against
MPI_Pack, typemap normalisation, and the argument checks of the flexible
calls (ncmpii_buftype_decode, dtype_decode.c:628-694)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLEX_CHECK = os.path.join(ROOT, "tests", "mpi", "flex_check")


def test_mpi_flatten_matches_mpi_pack():
    """pncx_mpi_type_flatten of 14 datatypes x 3 element types replayed as a
    host pack equals MPI_Pack byte for byte; mixed element types give
    NC_EMULTITYPES and MPI_BYTE gives NC_EBADTYPE."""
    if not os.path.exists(FLEX_CHECK):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "mpi")], check=True)
    r = subprocess.run([FLEX_CHECK, "flatten"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert r.stdout.count("ok flatten") == 3 * 14
    assert "ok error codes" in r.stdout


@pytest.mark.parametrize("disp,blen,ext,layout,nel", [
    ([0, 16, 32], [2, 2, 2], 48, 1, 6),          # uniform runs
    ([8, 0, 40], [2, 2, 3], 64, 2, 7),           # general table
    ([0, 8], [2, 2], 16, 0, 4),                  # runs merge into one contiguous run
    ([4, 0, 4], [0, 0, 3], 12, 0, 3),            # empty runs dropped
    ([], [], 0, 0, 0),                           # empty type
    ([12, 8, 4, 0], [1, 1, 1, 1], 16, 1, 4),     # descending, uniform negative stride
])
def test_type_commit_layouts(disp, blen, ext, layout, nel):
    from pnetcdf_amd import pncx
    d = pncx.DType(T.ITYPE_INT, disp, blen, ext)
    q = d.inq()
    assert (q["layout"], q["nelems"], q["extent"], q["itype"]) == (layout, nel, ext, T.ITYPE_INT)
    d.free()


def test_type_commit_rejects_bad_args():
    from pnetcdf_amd import pncx
    L = pncx.lib()
    h = ctypes.c_void_p()
    d = (ctypes.c_longlong * 2)(0, 8)
    bad = (ctypes.c_longlong * 2)(1, -1)
    assert L.pncx_type_commit(99, 2, d, d, 16, ctypes.byref(h)) == T.NC_EBADTYPE
    assert L.pncx_type_commit(T.ITYPE_INT, 2, d, bad, 16, ctypes.byref(h)) == T.NC_EINVAL
    assert L.pncx_type_commit(T.ITYPE_INT, -1, d, d, 16, ctypes.byref(h)) == T.NC_EINVAL


def test_flex_count_mismatch_before_device():
    """NC_EIOMISMATCH (dtype_decode.c:690) is an argument error: reported
    without touching a device."""
    from pnetcdf_amd import pncx
    dt = pncx.DType(T.ITYPE_INT, [0, 16], [2, 2], 32)      # 4 elements per copy
    xb = np.zeros(64, np.uint8)
    ub = np.zeros(256, np.uint8)
    with pytest.raises(pncx.PncxError) as e:
        pncx.putn_flex(5, T.NC_INT, xb, ub, [7], None, 2, dt)
    assert e.value.code == T.NC_EIOMISMATCH
    with pytest.raises(pncx.PncxError) as e:
        pncx.getn_flex(5, T.NC_INT, xb, ub, [8], None, 1, dt)
    assert e.value.code == T.NC_EIOMISMATCH
