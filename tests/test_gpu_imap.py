"""varm (imap) fused gather/scatter + conversion vs numpy gather + oracle (GPU).

Reference semantics: the user buffer is addressed through imap[] (element
strides, create_imaptype.c:25-139); MPI_Pack by that type then the
conversion (ncmpio_util.c:654-689, 716-765), or conversion then MPI_Unpack
(:842-966) for get.
"""
import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu


def offsets(count, imap):
    idx = np.indices(count).reshape(len(count), -1)
    return (idx * np.asarray(imap, np.int64)[:, None]).sum(0)


CASES = [
    ([4, 5, 6], [1, 4, 20]),          # transposed (Fortran-order) layout
    ([3, 7], [16, 2]),                 # padded rows, every other element
    ([2, 3, 4], [24, 8, 1]),           # already C order (no varm): contiguous path
    ([5, 1, 9], [100, 0, 11]),        # count 1 dim with imap 0
    ([1000, 3], [3, 1000]),            # tall-skinny transpose
    ([6], [5]),                        # 1-D strided
    # LDS-tiled transpose path (k_imap_tile): packed-fastest dim strided in the
    # user buffer, another dim (nearly) contiguous there
    ([37, 70], [1, 37]),              # 2-D Fortran order, partial edge tiles
    ([65, 20, 130], [2, 130, 2600]),  # padded (imap 2) fastest user dim, outer dim between
    ([3, 40, 50], [2000, 1, 40]),     # U in the middle, outer dim first
    ([16, 16], [1, 16]),              # exactly one tile
    ([200, 3, 130], [1, 200, 600]),   # 64 x 128 tiles: partial along U (72) and P (2)
    ([256, 2, 128], [1, 256, 512]),   # whole 64 x 128 tiles only
]
# every external type at least once: one code object per type (pncx_kern_xt.c)
PAIRS = [(T.NC_INT, T.ITYPE_DOUBLE), (T.NC_SHORT, T.ITYPE_FLOAT), (T.NC_DOUBLE, T.ITYPE_DOUBLE),
         (T.NC_BYTE, T.ITYPE_INT), (T.NC_UINT64, T.ITYPE_SCHAR), (T.NC_FLOAT, T.ITYPE_FLOAT),
         (T.NC_UBYTE, T.ITYPE_USHORT), (T.NC_USHORT, T.ITYPE_INT), (T.NC_UINT, T.ITYPE_DOUBLE),
         (T.NC_INT64, T.ITYPE_FLOAT)]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.mark.parametrize("count,imap", CASES)
@pytest.mark.parametrize("xt,it", PAIRS)
@pytest.mark.parametrize("where", ["host", "dev"])
def test_imap_put_get(torch_cuda, count, imap, xt, it, where):
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(sum(count) + xt * 11 + it)
    off = offsets(count, imap)
    n = off.size
    span = int(off.max()) + 1 if n else 0
    user = np.frombuffer(rng.integers(0, 256, span * T.ilen(it) + 8, dtype=np.uint8).tobytes(),
                         T.ITYPE_NP[it])[:span].copy()
    if np.issubdtype(user.dtype, np.floating):
        user = rng.standard_normal(span).astype(user.dtype) * 1e4
    fill = T.fill_bytes(xt, 42)
    # ---- put: gather + convert
    exp_x, exp_st = ora.putn(5, xt, user[off], it, fill)
    if where == "host":
        xb = np.zeros(n * T.xlen(xt), np.uint8)
        st = pncx.putn_imap(5, xt, xb, user, count, imap, it, fill)
        got_x = xb.tobytes()
    else:
        du = torch.from_numpy(user.view(np.uint8).copy()).cuda()
        dx = torch.zeros(max(n * T.xlen(xt), 16), dtype=torch.uint8, device="cuda")
        ds = torch.zeros(1, dtype=torch.int32, device="cuda")
        pncx.dev_putn_imap(5, xt, dx, du, count, imap, it, fill, ds)
        torch.cuda.synchronize()
        got_x, st = dx.cpu().numpy()[:n * T.xlen(xt)].tobytes(), int(ds.item())
    assert st == exp_st and got_x == exp_x
    # ---- get: convert + scatter (untouched user elements must survive)
    vals, gst = ora.getn(5, xt, exp_x, it)
    exp_user = user.copy()
    exp_user[off] = vals
    if where == "host":
        out = user.copy()
        st = pncx.getn_imap(5, xt, np.frombuffer(exp_x, np.uint8).copy(), out, count, imap, it)
    else:
        du = torch.from_numpy(user.view(np.uint8).copy()).cuda()
        dx = torch.from_numpy(np.frombuffer(exp_x + b"\0" * 16, np.uint8).copy()).cuda()
        ds = torch.zeros(1, dtype=torch.int32, device="cuda")
        pncx.dev_getn_imap(5, xt, dx, du, count, imap, it, ds)
        torch.cuda.synchronize()
        out = np.frombuffer(du.cpu().numpy().tobytes(), user.dtype)
        st = int(ds.item())
    assert st == gst
    assert out.tobytes() == exp_user.tobytes()


def test_imap_rejects_bad_args(torch_cuda):
    from pnetcdf_amd import pncx
    xb = np.zeros(64, np.uint8)
    ib = np.zeros(64, np.uint8)
    import ctypes
    lib = pncx.lib()
    cnt = (ctypes.c_longlong * 2)(2, -1)
    imp = (ctypes.c_longlong * 2)(1, 1)
    assert lib.pncx_putn_imap(5, T.NC_INT, xb.ctypes.data, ib.ctypes.data, 2, cnt, imp, T.ITYPE_INT, None) == T.NC_EINVAL
    assert lib.pncx_putn_imap(5, T.NC_INT, xb.ctypes.data, ib.ctypes.data, 17, cnt, imp, T.ITYPE_INT, None) == T.NC_EINVAL


@pytest.mark.parametrize("xt,it", [(T.NC_INT, T.ITYPE_DOUBLE), (T.NC_DOUBLE, T.ITYPE_DOUBLE),
                                   (T.NC_SHORT, T.ITYPE_FLOAT), (T.NC_UINT64, T.ITYPE_SCHAR)])
@pytest.mark.parametrize("ushift,xshift", [(0, 0), (1, 3), (0, 1), (2, 0)])
def test_imap_tile_alignment(torch_cuda, xt, it, ushift, xshift):
    """k_imap_tile takes its nontemporal full-tile path only when both device
    buffers are element-aligned; byte-shifted buffers take the checked loops.
    Full 64x64 tiles plus partial edges (130 x 3 x 70, Fortran order)."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    count, imap = [130, 3, 70], [1, 130, 390]
    rng = np.random.default_rng(ushift * 7 + xshift + xt * 3 + it)
    off = offsets(count, imap)
    n, span = off.size, int(off.max()) + 1
    isz, xsz = T.ilen(it), T.xlen(xt)
    user = np.frombuffer(rng.integers(0, 256, span * isz, dtype=np.uint8).tobytes(), T.ITYPE_NP[it]).copy()
    if np.issubdtype(user.dtype, np.floating):
        user = rng.standard_normal(span).astype(user.dtype) * 1e4
    fill = T.fill_bytes(xt, 42)
    exp_x, exp_st = ora.putn(5, xt, user[off], it, fill)
    ubuf = torch.zeros(span * isz + 16, dtype=torch.uint8, device="cuda")
    ubuf[ushift:ushift + span * isz] = torch.from_numpy(user.view(np.uint8).copy()).cuda()
    xbuf = torch.zeros(n * xsz + 16, dtype=torch.uint8, device="cuda")
    du, dx = ubuf[ushift:], xbuf[xshift:]
    ds = torch.zeros(1, dtype=torch.int32, device="cuda")
    pncx.dev_putn_imap(5, xt, dx, du, count, imap, it, fill, ds)
    torch.cuda.synchronize()
    assert int(ds.item()) == exp_st
    assert xbuf.cpu().numpy()[xshift:xshift + n * xsz].tobytes() == exp_x
    # get: convert + scatter back into a shifted copy; gaps keep their bytes
    vals, gst = ora.getn(5, xt, exp_x, it)
    exp_user = user.copy()
    exp_user[off] = vals
    ubuf[ushift:ushift + span * isz] = torch.from_numpy(user.view(np.uint8).copy()).cuda()
    ds.zero_()
    pncx.dev_getn_imap(5, xt, dx, du, count, imap, it, ds)
    torch.cuda.synchronize()
    assert int(ds.item()) == gst
    assert ubuf.cpu().numpy()[ushift:ushift + span * isz].tobytes() == exp_user.view(np.uint8).tobytes()


# the transposes whose last two dimensions are tiled as one (U is not P-1):
# 2000-byte packed rows, a 4-D request with an outer dim between U and
# (P-1, P), count[P] = 16 (the smallest: a lane's two-row step wraps), a
# padded U (imap 2), and partial tiles at the end of the merged rows
MERGE_CASES = [
    ([130, 9, 250], [1, 130, 1170]),
    ([130, 5, 7, 70], [1, 130, 650, 4550]),
    ([150, 33, 16], [1, 150, 4950]),
    ([65, 11, 37], [2, 130, 1430]),
    ([129, 3, 19], [1, 129, 387]),
]


@pytest.mark.parametrize("count,imap", MERGE_CASES)
@pytest.mark.parametrize("xt,it", [(T.NC_INT, T.ITYPE_DOUBLE), (T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_UINT64, T.ITYPE_SCHAR)])
@pytest.mark.parametrize("merge", ["1", "0"])
@pytest.mark.parametrize("order", [0, 1], ids=["rowmajor", "diagonal"])
def test_imap_tile_merged_dims(torch_cuda, count, imap, xt, it, merge, order, knob):
    """k_imap_tile with the last two dimensions tiled as one virtual row
    (default) and tiled P alone (PNCX_XPOSE_MERGE=0), tiles in row-major or
    diagonal order (PNCX_XPOSE_ORDER): put and get against a numpy
    gather/scatter + the oracle, on device buffers."""
    knob("XPOSE_MERGE", merge)
    knob("XPOSE_ORDER", order)
    test_imap_put_get(torch_cuda, count, imap, xt, it, "dev")


@pytest.mark.parametrize("xt,it", [(T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_INT, T.ITYPE_DOUBLE), (T.NC_SHORT, T.ITYPE_FLOAT)])
def test_imap_tile_channel_skew(torch_cuda, xt, it):
    """a packed U stride just under a multiple of 2 MiB (1024 x 254 doubles
    = 2^21 - 2^14 B, as the x 254 benchmark shape) takes the skewed tile
    order by default (p0 shifted by 8 tiles per u tile on put, 32 on get);
    the narrower external types give strides off that band and keep the
    default order -- both against the oracle"""
    test_imap_put_get(torch_cuda, [16, 1024, 254], [1, 16, 16 * 1024], xt, it, "dev")


# 2-D transposes (U = P - 1) with tile grids wider than tall, taller than
# wide and partial tiles on both edges, in both tile orders
XPOSE2D_CASES = [([300, 70], [1, 300]), ([70, 300], [1, 70]), ([257, 129], [1, 257]), ([128, 64], [1, 128])]


@pytest.mark.parametrize("count,imap", XPOSE2D_CASES)
@pytest.mark.parametrize("order", [0, 1], ids=["rowmajor", "diagonal"])
def test_imap_tile_2d_orders(torch_cuda, count, imap, order, knob):
    knob("XPOSE_ORDER", order)
    for xt, it in ((T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_SHORT, T.ITYPE_FLOAT)):
        test_imap_put_get(torch_cuda, count, imap, xt, it, "dev")


# varm with a contiguous fastest dimension holding whole 16-byte vectors
# (k_imap_rows): padded rows of a 3-D interior, a 2-D row gather, and a
# count that is not a multiple of the vector (falls back to k_imap)
ROW_CASES = [
    ([6, 5, 34], [1000, 40, 1]),
    ([9, 18], [20, 1]),
    ([7, 13], [16, 1]),
    ([3, 4, 64], [4096, 70, 1]),
]


@pytest.mark.parametrize("count,imap", ROW_CASES)
@pytest.mark.parametrize("xt,it", [(T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_INT, T.ITYPE_DOUBLE), (T.NC_SHORT, T.ITYPE_INT),
                                   (T.NC_BYTE, T.ITYPE_UCHAR), (T.NC_FLOAT, T.ITYPE_FLOAT)])
@pytest.mark.parametrize("rows", ["1", "0"])
def test_imap_contiguous_rows(torch_cuda, count, imap, xt, it, rows, knob):
    """varm rows contiguous in the user buffer, a vector per lane
    (PNCX_IMAP_ROWS=1, default) or an element per lane (0): put and get
    against a numpy gather/scatter + the oracle, host and device buffers"""
    knob("IMAP_ROWS", rows)
    for where in ("host", "dev"):
        test_imap_put_get(torch_cuda, count, imap, xt, it, where)
