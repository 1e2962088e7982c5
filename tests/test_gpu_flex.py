"""Derived user-buffer datatypes (flexible API) vs numpy pack + the CPU oracle (GPU).

Reference semantics (ncmpio_pack_xbuf, ncmpio_util.c:620-689, 716-765; unpack
:842-966): MPI_Pack the bufcount copies of the buftype into a contiguous lbuf,
then the imap type, then convert; for get, convert then MPI_Unpack (bytes of
the user buffer between the runs are untouched).  The typemap model here is
numpy: element k of copy c sits at c*extent + disp[b] + (k - pre[b])*isize.
The kernels fuse that gather/scatter into the conversion (pncx_kern.hpp
tmap_byte).  The MPI side (flattening real MPI datatypes, and the whole
flexible file path vs MPI_Pack/Unpack) is tests/mpi/flex_check.c.
"""
import os
import subprocess
import zlib

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def elem_offsets(disp, blocklen, extent, bufcount, isz):
    """byte offset of every packed element (MPI_Pack order)"""
    one = np.concatenate([d + isz * np.arange(b, dtype=np.int64) for d, b in zip(disp, blocklen)]
                         or [np.zeros(0, np.int64)])
    return (np.arange(bufcount, dtype=np.int64)[:, None] * extent + one[None, :]).reshape(-1)


def imap_offsets(count, imap):
    idx = np.indices(count).reshape(len(count), -1)
    return (idx * np.asarray(imap, np.int64)[:, None]).sum(0)


# (name, disp in elements, blocklen, extent in elements, bufcount) -- layout the commit must pick
TYPES = [
    ("vector", [0, 4, 8], [2, 2, 2], 12, 2, 1),
    ("indexed_irregular", [7, 0, 11, 3], [2, 1, 3, 1], 14, 2, 2),
    ("contig_offset", [3], [10], 10, 3, 0),
    ("negative_disp", [4, -2, 9], [2, 1, 2], 12, 1, 2),
    ("single_block_resized", [0], [3], 7, 4, 1),
    ("runs_merge", [0, 2, 5], [2, 3, 1], 9, 2, 1),     # the three runs merge into one: uniform
    ("descending", [9, 6, 3, 0], [1, 1, 1, 1], 10, 3, 1),
]
PAIRS = [(T.NC_INT, T.ITYPE_INT), (T.NC_FLOAT, T.ITYPE_DOUBLE), (T.NC_SHORT, T.ITYPE_INT),
         (T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_BYTE, T.ITYPE_SCHAR), (T.NC_INT64, T.ITYPE_LONGLONG),
         (T.NC_UBYTE, T.ITYPE_FLOAT)]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def user_values(rng, it, nbytes):
    isz = T.ilen(it)
    n = nbytes // isz
    if np.issubdtype(np.dtype(T.ITYPE_NP[it]), np.floating):
        v = (rng.standard_normal(n) * 4e4).astype(T.ITYPE_NP[it])
    else:
        v = np.frombuffer(rng.integers(0, 256, n * isz, dtype=np.uint8).tobytes(), T.ITYPE_NP[it]).copy()
        if isz >= 4:
            v = (v % 70000 - 35000).astype(T.ITYPE_NP[it])    # some out of range for NC_SHORT
    return v.view(np.uint8)


def run_case(torch, where, xt, it, disp_el, blocklen, ext_el, bufcount, count, imap, seed):
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(seed)
    isz, xsz = T.ilen(it), T.xlen(xt)
    disp = [d * isz for d in disp_el]
    offs = elem_offsets(disp, blocklen, ext_el * isz, bufcount, isz)
    lo = int(offs.min()) if offs.size else 0
    hi = int(offs.max()) + isz if offs.size else 0
    base = -lo + 16                                       # buffer origin inside the array
    ub = user_values(rng, it, base + hi + 16)
    n = offs.size
    if count is None:
        count, imap = [n], None
    jm = np.arange(n) if imap is None else imap_offsets(count, imap)
    src = (base + offs[jm])[:, None] + np.arange(isz)[None, :]
    packed = ub[src.reshape(-1)].view(T.ITYPE_NP[it])
    fill = T.fill_bytes(xt, 42)
    exp_x, exp_st = ora.putn(5, xt, packed, it, fill)
    dt = pncx.DType(it, disp, blocklen, ext_el * isz)
    # ---- put
    if where == "host":
        xb = np.zeros(n * xsz, np.uint8)
        st = pncx.putn_flex(5, xt, xb, ub, count, imap, bufcount, dt, fill, base=base)
        got_x = xb.tobytes()
    else:
        du = torch.from_numpy(ub.copy()).cuda()
        dx = torch.zeros(max(n * xsz, 16), dtype=torch.uint8, device="cuda")
        ds = torch.zeros(1, dtype=torch.int32, device="cuda")
        pncx.dev_putn_flex(5, xt, dx, du, count, imap, bufcount, dt, fill, ds, base=base)
        torch.cuda.synchronize()
        got_x, st = dx.cpu().numpy()[:n * xsz].tobytes(), int(ds.item())
    assert st == exp_st and got_x == exp_x
    # ---- get: convert + unpack; everything else in the user buffer survives
    vals, gst = ora.getn(5, xt, exp_x, it)
    exp_ub = ub.copy()
    exp_ub[src.reshape(-1)] = np.ascontiguousarray(vals).view(np.uint8)
    if where == "host":
        out = ub.copy()
        st = pncx.getn_flex(5, xt, np.frombuffer(exp_x, np.uint8).copy(), out, count, imap, bufcount, dt, base=base)
    else:
        du = torch.from_numpy(ub.copy()).cuda()
        dx = torch.from_numpy(np.frombuffer(exp_x + b"\0" * 16, np.uint8).copy()).cuda()
        ds = torch.zeros(1, dtype=torch.int32, device="cuda")
        pncx.dev_getn_flex(5, xt, dx, du, count, imap, bufcount, dt, ds, base=base)
        torch.cuda.synchronize()
        out, st = du.cpu().numpy(), int(ds.item())
    assert st == gst
    assert out.tobytes() == exp_ub.tobytes()
    return dt


@pytest.mark.parametrize("tname,disp,blen,ext,bufcount,layout", TYPES)
@pytest.mark.parametrize("xt,it", PAIRS)
@pytest.mark.parametrize("where", ["host", "dev"])
def test_flex_typemap(torch_cuda, tname, disp, blen, ext, bufcount, layout, xt, it, where):
    dt = run_case(torch_cuda, where, xt, it, disp, blen, ext, bufcount, None, None,
                  seed=zlib.crc32(f"{tname}/{xt}/{it}".encode()))
    assert dt.inq()["layout"] == layout


@pytest.mark.parametrize("where", ["host", "dev"])
def test_flex_with_imap(torch_cuda, where):
    # 12 packed elements (2 copies x 6) read through a transposing imap
    run_case(torch_cuda, where, T.NC_FLOAT, T.ITYPE_DOUBLE, [7, 0, 11, 3], [2, 1, 2, 1], 14, 2, [3, 4], [1, 3], 7)
    run_case(torch_cuda, where, T.NC_INT, T.ITYPE_INT, [0, 4, 8], [2, 2, 2], 12, 2, [4, 3], [1, 4], 8)


@pytest.mark.parametrize("where", ["host", "dev"])
def test_flex_large_table(torch_cuda, where):
    # 2^16 irregular runs (binary-search layout) x 4 copies, ~1M elements
    rng = np.random.default_rng(5)
    nb = 1 << 16
    blen = rng.integers(1, 8, nb)
    gaps = rng.integers(0, 5, nb)
    disp = np.concatenate([[0], np.cumsum(blen + gaps)[:-1]]).astype(np.int64)
    ext = int(disp[-1] + blen[-1] + 3)
    dt = run_case(torch_cuda, where, T.NC_INT, T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(), ext, 4,
                  None, None, 9)
    assert dt.inq()["layout"] == 2


@pytest.mark.parametrize("where", ["host", "dev"])
def test_flex_table_search_path(torch_cuda, where, knob):
    """short-run tables normally get a per-element offset map at commit
    (tmode 4); with the map disabled the same cases take the chunk-indexed
    table search (tmode 2)"""
    knob("TOFF_MAX_ELEMS", "0")
    for tname, disp, blen, ext, bufcount, layout in TYPES:
        if layout == 2:
            dt = run_case(torch_cuda, where, T.NC_SHORT, T.ITYPE_INT, disp, blen, ext, bufcount, None, None,
                          seed=zlib.crc32(tname.encode()))
            assert dt.inq()["layout"] == 2
    run_case(torch_cuda, where, T.NC_FLOAT, T.ITYPE_DOUBLE, [7, 0, 11, 3], [2, 1, 2, 1], 14, 2, [3, 4], [1, 3], 7)
    rng = np.random.default_rng(6)
    nb = 1 << 14
    blen = rng.integers(1, 8, nb)
    gaps = rng.integers(0, 5, nb)
    disp = np.concatenate([[0], np.cumsum(blen + gaps)[:-1]]).astype(np.int64)
    run_case(torch_cuda, where, T.NC_INT, T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(), int(disp[-1] + blen[-1] + 3),
             3, None, None, 13)


@pytest.mark.parametrize("where", ["host", "dev"])
@pytest.mark.parametrize("map16", ["-1", "8", "16", "0"], ids=["auto4", "8", "16", "32"])
@pytest.mark.parametrize("gap", [5, 16, 17, 3000])
@pytest.mark.parametrize("tgap", ["-1", "0"], ids=["tgap", "imap"])
def test_flex_offset_map_widths(torch_cuda, where, map16, gap, tgap, knob):
    """short-run tables get a 4-bit gap-step map (tmode 7) when offsets rise
    through every 64-element chunk with gaps of at most 15 elements, else an
    8-bit gap map (tmode 6) with under 256 gap elements per chunk, else a
    16-bit offset map (a base per chunk, tmode 5) when every chunk spans
    under 64 KiB, else the 32-bit map (tmode 4); PNCX_TOFF16=8 / 16 start at
    8 / 16 bits, 0 forces 32.  Gaps of 0..15 fit the nibbles exactly, 0..16
    do not; gaps of up to 3000 elements make chunks span ~1.5 MiB of doubles
    (32-bit map by necessity); partial last chunk and several copies
    included; runs in falling order take the wider maps.  PNCX_TGAP=0 moves
    the 8-bit map from the wave-per-chunk kernel (k_tgap) to k_imap; the
    4-bit map always takes k_tgap over whole copies."""
    knob("TOFF16", map16)
    knob("TGAP", tgap)
    rng = np.random.default_rng(gap + abs(int(map16)))
    nb = 5000
    blen = rng.integers(1, 8, nb)
    gaps = rng.integers(0, gap, nb)
    disp = np.concatenate([[0], np.cumsum(blen + gaps)[:-1]]).astype(np.int64)
    dt = run_case(torch_cuda, where, T.NC_FLOAT, T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(),
                  int(disp[-1] + blen[-1] + 5), 3, None, None, 21)
    assert dt.inq()["layout"] == 2
    # the same runs in falling order: offsets drop inside chunks
    run_case(torch_cuda, where, T.NC_FLOAT, T.ITYPE_DOUBLE, disp[::-1].tolist(), blen[::-1].tolist(),
             int(disp[-1] + blen[-1] + 5), 2, None, None, 23)
    # through a transposing imap as well (imap offset -> typemap stage)
    run_case(torch_cuda, where, T.NC_INT, T.ITYPE_INT, [9, 0, 20, 3, 40], [2, 1, 5, 1, 3], 50, 4, [12, 4], [1, 12], 22)


GAP_SHAPES = [
    ([0, 3, 9], [2, 1, 3], 14, 300),                 # tn 6 < one chunk, many copies
    (list(range(0, 128, 2)), [1] * 64, 130, 7),      # tn exactly 64, every other element
    (list(range(0, 130, 2)), [1] * 65, 131, 5),      # tn 65: a one-element second chunk
    ([0, 30, 62], [15, 17, 10], 80, 9),              # gaps of exactly 15 elements fit the nibbles
]


@pytest.mark.parametrize("where", ["host", "dev"])
@pytest.mark.parametrize("shape", range(len(GAP_SHAPES)))
@pytest.mark.parametrize("xt,it", [(T.NC_SHORT, T.ITYPE_INT), (T.NC_INT, T.ITYPE_SCHAR), (T.NC_DOUBLE, T.ITYPE_DOUBLE)])
def test_flex_gap_map_edges(torch_cuda, where, shape, xt, it, knob):
    """the 4-bit map on k_tgap at its edges: typemaps shorter than a chunk
    with hundreds of copies, exactly one chunk, one chunk and one element,
    gaps of exactly 15 elements; NC_ERANGE both ways (int -> NC_SHORT on put,
    NC_INT -> schar on get) and a plain swap; against the oracle"""
    knob("TOFF16", "-1")
    disp, blen, ext, bufcount = GAP_SHAPES[shape]
    run_case(torch_cuda, where, xt, it, disp, blen, ext, bufcount, None, None, 50 + shape)


@pytest.mark.parametrize("where", ["host", "dev"])
@pytest.mark.parametrize("map16", ["-1", "8"], ids=["map4", "map8"])
def test_flex_gap_map_through_imap(torch_cuda, where, map16, knob):
    """rising short runs under a transposing imap: the 4-bit map is decoded
    per element (a masked nibble sum over the chunk's 32 bytes) by k_imap,
    the 8-bit map by its lookup; 150 runs span several chunks and end in a
    partial one"""
    knob("TOFF16", map16)
    rng = np.random.default_rng(31)
    nb = 150
    blen = rng.integers(1, 8, nb)
    gaps = rng.integers(0, 16, nb)
    disp = np.concatenate([[3], 3 + np.cumsum(blen + gaps)[:-1]]).astype(np.int64)
    tn = int(blen.sum())
    run_case(torch_cuda, where, T.NC_INT, T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(),
             int(disp[-1] + blen[-1] + 2), 6, [6, tn], [1, 6], 41)


@pytest.mark.parametrize("where", ["host", "dev"])
@pytest.mark.parametrize("imap", [False, True])
def test_flex_long_runs(torch_cuda, where, imap):
    """runs of 50..1500 elements: one wave per run piece (k_tmap_runs, runs
    split into pieces of <= 512 at commit); through an imap the same piece
    table is searched per element"""
    rng = np.random.default_rng(11)
    nb = 300
    blen = rng.integers(50, 1500, nb)
    gaps = rng.integers(0, 40, nb)
    disp = np.concatenate([[5], 5 + np.cumsum(blen + gaps)[:-1]]).astype(np.int64)
    ext = int(disp[-1] + blen[-1] + 7)
    n = int(blen.sum()) * 3
    count, im = ([3, n // 3], [1, 3]) if imap else (None, None)
    dt = run_case(torch_cuda, where, T.NC_SHORT, T.ITYPE_FLOAT, disp.tolist(), blen.tolist(), ext, 3,
                  count, im, 12)
    assert dt.inq()["layout"] == 2


@pytest.mark.parametrize("where", ["host", "dev"])
@pytest.mark.parametrize("blen,imap", [(64, False), (256, False), (300, False), (4096, False), (5000, False),
                                       (300, True)])
def test_flex_uniform_long_runs(torch_cuda, where, blen, imap):
    """uniform runs of 256..4096 elements in packed order go one wave per run
    (k_tmap_runs, tmode 1); shorter or longer runs, or an imap, take k_imap"""
    nb = 3000 if blen <= 64 else 40
    disp = (np.arange(nb) * (blen + 16) + 3).tolist()
    n = nb * blen * 2
    count, im = ([2, n // 2], [1, 2]) if imap else (None, None)
    dt = run_case(torch_cuda, where, T.NC_FLOAT, T.ITYPE_DOUBLE, disp, [blen] * nb, nb * (blen + 16) + 5, 2,
                  count, im, 14 + blen)
    assert dt.inq()["layout"] == 1


@pytest.mark.parametrize("where", ["host", "dev"])
def test_flex_large_uniform(torch_cuda, where):
    # vector(2^18 blocks of 3, stride 5) x 2 copies
    nb = 1 << 18
    disp = (np.arange(nb) * 5).tolist()
    dt = run_case(torch_cuda, where, T.NC_DOUBLE, T.ITYPE_DOUBLE, disp, [3] * nb, 5 * nb + 1, 2, None, None, 10)
    assert dt.inq()["layout"] == 1


def test_flex_mpi_file_parity(tmp_path):
    """The whole flexible file path with real MPI datatypes (contiguous,
    (h)vector, (h)indexed, (h)indexed_block, struct, subarray C/Fortran,
    resized, nested, dup, darray) x 4 conversions: derived-type put/iput and
    get/iget equal MPI_Pack + contiguous put and contiguous get + MPI_Unpack."""
    exe = os.path.join(ROOT, "tests", "mpi", "flex_check")
    assert os.path.exists(exe), "tests/mpi/flex_check not built (run __graft_entry__.build())"
    r = subprocess.run([exe, "file", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "file: 0 failure(s)" in r.stdout
    assert r.stdout.count("ok file") == 4 * 14


@pytest.mark.parametrize("xt,it", [(T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_SHORT, T.ITYPE_INT)])
def test_flex_short_runs_many_steps(torch_cuda, xt, it):
    """the 16-bit-map short-run path with 2^17 runs x 12 copies: every lane
    takes several grid-stride steps and the last one is ragged"""
    rng = np.random.default_rng(0x70FF)
    nb = 1 << 17
    blen = rng.integers(1, 8, nb)
    gaps = rng.integers(0, 5, nb)
    disp = np.concatenate([[0], np.cumsum(blen + gaps)[:-1]]).astype(np.int64)
    dt = run_case(torch_cuda, "dev", xt, it, disp.tolist(), blen.tolist(), int(disp[-1] + blen[-1] + 2), 12,
                  None, None, 31)
    assert dt.inq()["layout"] == 2


@pytest.mark.parametrize("urun", ["1", "0"])
@pytest.mark.parametrize("blen,gap", [(2, 2), (64, 16), (300, 4), (3, 1), (1, 1), (5, 11)])
@pytest.mark.parametrize("xt,it", [(T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_FLOAT, T.ITYPE_DOUBLE),
                                   (T.NC_SHORT, T.ITYPE_INT), (T.NC_INT, T.ITYPE_SHORT)])
@pytest.mark.parametrize("where", ["host", "dev"])
def test_flex_uniform_vector_runs(torch_cuda, where, xt, it, blen, gap, urun, knob):
    """uniform runs whose lengths hold whole 16-byte vectors, 16-byte aligned,
    over a contiguous count: one vector per lane (k_urun; PNCX_URUN=0 takes
    k_imap / k_tmap_runs).  Blocks that do not divide into vectors (1, 3, 5;
    2 of NC_FLOAT <- double) fall back to k_imap either way.  3 copies,
    NC_ERANGE from int -> NC_SHORT."""
    knob("URUN", urun)
    nb = 4096 if blen <= 64 else 64
    disp = (np.arange(nb) * (blen + gap)).tolist()
    dt = run_case(torch_cuda, where, xt, it, disp, [blen] * nb, nb * (blen + gap), 3, None, None, 40 + blen)
    assert dt.inq()["layout"] == 1


@pytest.mark.parametrize("tmap_imap", ["1", "0"])
@pytest.mark.parametrize("xt,it", [(T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.NC_INT, T.ITYPE_DOUBLE), (T.NC_SHORT, T.ITYPE_INT),
                                   (T.NC_FLOAT, T.ITYPE_FLOAT), (T.NC_BYTE, T.ITYPE_UCHAR)])
@pytest.mark.parametrize("where", ["host", "dev"])
@pytest.mark.parametrize("ghost", [1, 2])
def test_flex_lattice_subarray(torch_cuda, where, xt, it, tmap_imap, ghost, knob):
    """a 3-D subarray buftype (interior of a ghosted block: equal runs on a
    2-level lattice) x 2 copies: with PNCX_TMAP_IMAP=1 (default) it runs as a
    4-D varm over the first run (k_imap_rows) when its rows hold whole
    vectors, else through the run-piece kernel; both against numpy + oracle"""
    knob("TMAP_IMAP", tmap_imap)
    L = (9, 10, 12)
    z, y = np.meshgrid(np.arange(L[0] - 2 * ghost), np.arange(L[1] - 2 * ghost), indexing="ij")
    disp = (((z + ghost) * L[1] * L[2] + (y + ghost) * L[2] + ghost)).reshape(-1).tolist()
    blen = [L[2] - 2 * ghost] * len(disp)
    dt = run_case(torch_cuda, where, xt, it, disp, blen, L[0] * L[1] * L[2], 2, None, None, 60 + ghost)
    assert dt.inq()["layout"] == 2
