"""Parity of the HIP path against the CPU oracle and the golden fixtures (GPU).

Bar: bit-exact outputs and identical status for every (xtype, itype) pair,
both directions, through the C-ABI (host-buffer and device-buffer entry
points).  Cross-type float casts are also bit-exact here (stricter than the
north star's 1-ulp allowance): tolerance = 0 ulp.
"""
import ctypes
import os

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from tests import reftests
from tests.converters import HipDevConv, HipHostConv, OracleConv

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "edge_vectors.npz"))


def pairs():
    for xt in T.NUMERIC_XTYPES:
        for it in T.NUMERIC_ITYPES:
            k = f"{T.XNAME[xt]}_{T.INAME[it]}"
            yield 5, xt, it, k
            if xt == T.NC_BYTE and it == T.ITYPE_UCHAR:
                yield 2, xt, it, k + "_cdf2"


PAIRS = list(pairs())


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    from pnetcdf_amd import pncx
    assert pncx.device_count() >= 1
    return torch


@pytest.fixture(scope="module", params=["host", "dev"])
def conv(request, torch_cuda):
    return HipHostConv() if request.param == "host" else HipDevConv()


# ------------------------------------------------------------------ golden
@pytest.mark.parametrize("cdf,xt,it,k", PAIRS, ids=[p[3] for p in PAIRS])
def test_golden_edges(conv, cdf, xt, it, k):
    res, st = conv.getn(cdf, xt, GOLD[f"get_{k}_in"].tobytes(), it)
    assert st == GOLD[f"get_{k}_st"][0]
    exp = GOLD[f"get_{k}_out"].tobytes()
    got = res.tobytes()
    if got != exp:
        e = np.frombuffer(exp, T.ITYPE_NP[it])
        bad = np.nonzero(res.view(np.uint8).reshape(res.size, -1).tobytes() != exp)[0]
        idx = [i for i in range(res.size) if res[i:i + 1].tobytes() != e[i:i + 1].tobytes()][:5]
        xin = np.frombuffer(GOLD[f"get_{k}_in"].tobytes(), T.XTYPE_BE[xt])
        pytest.fail(f"get mismatch at {idx}: in {[xin[i] for i in idx]} got {[res[i] for i in idx]} "
                    f"exp {[e[i] for i in idx]} ({len(bad)})")
    iin = np.frombuffer(GOLD[f"put_{k}_in"].tobytes(), T.ITYPE_NP[it])
    for tag, fill in (("dflt", T.fill_bytes(xt)), ("user", T.fill_bytes(xt, 99)), ("null", None)):
        xb, st = conv.putn(cdf, xt, iin, it, fill, xinit=GOLD[f"put_{k}_xinit"].tobytes())
        assert st == GOLD[f"put_{k}_{tag}_st"][0], tag
        exp = GOLD[f"put_{k}_{tag}_out"].tobytes()
        if xb != exp:
            xs = T.xlen(xt)
            idx = [i for i in range(iin.size) if xb[i * xs:(i + 1) * xs] != exp[i * xs:(i + 1) * xs]][:5]
            pytest.fail(f"put {tag} mismatch at {idx}: in {[iin[i] for i in idx]} got "
                        f"{[xb[i*xs:(i+1)*xs].hex() for i in idx]} exp {[exp[i*xs:(i+1)*xs].hex() for i in idx]}")


# ------------------------------------------------- random bits vs the oracle
@pytest.mark.parametrize("xt", T.NUMERIC_XTYPES, ids=[T.XNAME[x] for x in T.NUMERIC_XTYPES])
def test_random_bits_vs_oracle(conv, xt):
    ora = OracleConv()
    rng = np.random.default_rng(0x5EED0000 + xt)
    for it in T.NUMERIC_ITYPES:
        for n in (1, 7, 33, 4099):
            raw = rng.integers(0, 256, n * 8, dtype=np.uint8)
            ib = np.frombuffer(raw.tobytes(), T.ITYPE_NP[it])[:n].copy()
            fill = T.fill_bytes(xt, 77)
            assert conv.putn(5, xt, ib, it, fill) == ora.putn(5, xt, ib, it, fill), (T.INAME[it], n)
            xr = rng.integers(0, 256, n * T.xlen(xt), dtype=np.uint8).tobytes()
            g, sg = conv.getn(5, xt, xr, it)
            o, so = ora.getn(5, xt, xr, it)
            assert sg == so and g.tobytes() == o.tobytes(), (T.INAME[it], n)


@pytest.mark.parametrize("u", [1, 2, 4])
def test_tiles_per_block_vs_oracle(torch_cuda, u, knob):
    """The direct-shape kernels with 1, 2 or 4 tiles per block (k_tile /
    k_tile_u, PNCX_TILE_U; the default is 2 for the 2:1 widening tiles and 1
    otherwise): every pair both ways on random bits, with tile counts that
    are not multiples of u and scalar tails."""
    knob("TILE_U", str(u))
    dev, ora = HipDevConv(), OracleConv()
    rng = np.random.default_rng(0x711E + u)
    for xt in T.NUMERIC_XTYPES:
        for it in T.NUMERIC_ITYPES:
            for n in (4099, 100003):
                raw = rng.integers(0, 256, n * 8, dtype=np.uint8)
                ib = np.frombuffer(raw.tobytes(), T.ITYPE_NP[it])[:n].copy()
                fill = T.fill_bytes(xt, 77)
                assert dev.putn(5, xt, ib, it, fill) == ora.putn(5, xt, ib, it, fill), (T.INAME[it], n)
                xr = rng.integers(0, 256, n * T.xlen(xt), dtype=np.uint8).tobytes()
                g, sg = dev.getn(5, xt, xr, it)
                o, so = ora.getn(5, xt, xr, it)
                assert sg == so and g.tobytes() == o.tobytes(), (T.XNAME[xt], T.INAME[it], n)


# ------------------------------------- the reference's own test expectations
@pytest.mark.parametrize("cdf", [2, 5])
def test_reference_nc_test(conv, cdf):
    fails = []
    for xt in T.NUMERIC_XTYPES:
        if cdf < 5 and xt in (T.NC_UBYTE, T.NC_USHORT, T.NC_UINT, T.NC_INT64, T.NC_UINT64):
            continue
        for it in T.NUMERIC_ITYPES:
            fails += [f"{T.XNAME[xt]}/{T.INAME[it]}: {m}" for m in reftests.nc_test_put_get(conv, cdf, xt, it)]
    assert not fails, "\n".join(fails[:20])


def test_reference_test_erange(conv):
    fails = reftests.test_erange_cases(conv)
    assert not fails, "\n".join(fails)


@pytest.mark.parametrize("cdf", [2, 5])
def test_reference_erange_fill(conv, cdf):
    fails = reftests.erange_fill_cases(conv, cdf)
    assert not fails, "\n".join(fails)


# ------------------------------------------------------------------- swaps
@pytest.mark.parametrize("esize", [2, 3, 4, 8, 16])
@pytest.mark.parametrize("n", [0, 1, 15, 17, 1000, 100003])
def test_host_in_swapn(torch_cuda, esize, n):
    from oracle import oracle as O
    from pnetcdf_amd import pncx
    rng = np.random.default_rng(esize * 1000 + n)
    buf = rng.integers(0, 256, n * esize, dtype=np.uint8)
    ref = buf.copy()
    O.in_swapn(ref, esize)
    pncx.in_swapn(buf, n, esize)
    assert np.array_equal(buf, ref)


@pytest.mark.parametrize("kind", ["pageable", "pageable_unaligned", "torch_pinned", "registered"])
def test_host_large_pinned_paths(torch_cuda, kind):
    """Host buffers >= 64 MiB are pinned for the call (hipHostRegister) and
    unpinned after; already-pinned buffers are used as they are.  Multi-chunk
    sizes, repeated calls (register/unregister cycles), swap + getn + putn."""
    from pnetcdf_amd import pncx
    n = (96 << 20) // 8 + 5
    rng = np.random.default_rng(0x9127)
    if kind == "torch_pinned":
        raw = torch_cuda.empty(n * 8 + 16, dtype=torch_cuda.uint8, pin_memory=True).numpy()
        raw[:] = rng.integers(0, 256, raw.size, dtype=np.uint8)
        buf = raw[:n * 8]
    else:
        raw = rng.integers(0, 256, n * 8 + 16, dtype=np.uint8)
        buf = raw[3:3 + n * 8] if kind == "pageable_unaligned" else raw[:n * 8]
    if kind == "registered":
        pncx.host_register(raw)
        pncx.host_register(raw)          # already pinned: still NC_NOERR
    orig = buf.copy()
    for _ in range(2):
        pncx.in_swapn(buf, n, 8)
        assert np.array_equal(buf.view(np.uint8).reshape(-1, 8), orig.reshape(-1, 8)[:, ::-1])
        pncx.in_swapn(buf, n, 8)
        assert np.array_equal(buf, orig)
    # NC_INT (big-endian) -> double, then double -> NC_INT with ERANGE fill
    m = buf.size // 4
    out = np.empty(m, np.float64)
    st = pncx.getn(5, T.NC_INT, buf, out, m, T.ITYPE_DOUBLE)
    assert st == T.NC_NOERR
    assert np.array_equal(out, np.frombuffer(buf.tobytes(), ">i4").astype(np.float64))
    out[::1000] = 1e300
    xb = np.empty(m * 4, np.uint8)
    st = pncx.putn(5, T.NC_INT, xb, out, m, T.ITYPE_DOUBLE, T.fill_bytes(T.NC_INT))
    assert st == T.NC_ERANGE
    exp = np.frombuffer(buf.tobytes(), ">i4").copy()
    exp[::1000] = T.XTYPE_FILL[T.NC_INT]
    assert np.array_equal(np.frombuffer(xb.tobytes(), ">i4"), exp)
    if kind == "registered":
        pncx.host_unregister(raw)


@pytest.mark.parametrize("esize", [2, 4, 8])
@pytest.mark.parametrize("offset", [0, 1, 2, 4, 8, 12])
def test_dev_swap_offsets(torch_cuda, esize, offset):
    """Element-aligned and misaligned device slabs (head/tail/scalar paths)."""
    torch = torch_cuda
    from oracle import oracle as O
    from pnetcdf_amd import pncx
    n = 4096 + 5
    rng = np.random.default_rng(offset)
    raw = rng.integers(0, 256, n * esize + 64, dtype=np.uint8)
    d = torch.from_numpy(raw.copy()).cuda()
    view = d[offset:offset + n * esize]
    lib = pncx.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.pncx_dev_in_swapn(ctypes.c_void_p(view.data_ptr()), n, esize, stream) == 0
    torch.cuda.synchronize()
    ref = raw.copy()
    seg = ref[offset:offset + n * esize]
    O.in_swapn(seg, esize)
    assert np.array_equal(d.cpu().numpy(), ref)


def test_dev_swapn_out_of_place(torch_cuda):
    torch = torch_cuda
    from pnetcdf_amd import pncx
    n = 1 << 20
    a = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda")
    b = torch.empty_like(a)
    pncx.dev_swapn(b, a, n, 8)
    torch.cuda.synchronize()
    assert torch.equal(b.view(torch.uint8).view(-1, 8).flip(1).reshape(-1), a.view(torch.uint8))


def test_misaligned_conversion(torch_cuda):
    """Pointers that cannot be co-aligned to 16 B take the scalar kernel."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    lib = pncx.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    n = 1000
    rng = np.random.default_rng(3)
    xr = rng.integers(0, 256, 4 * n, dtype=np.uint8)
    dx = torch.zeros(4 * n + 64, dtype=torch.uint8, device="cuda")
    dx[1:1 + 4 * n] = torch.from_numpy(xr).cuda()
    di = torch.zeros(8 * n + 64, dtype=torch.uint8, device="cuda")
    ds = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = lib.pncx_dev_getn(5, T.NC_INT, ctypes.c_void_p(dx.data_ptr() + 1), ctypes.c_void_p(di.data_ptr() + 3),
                           n, T.ITYPE_DOUBLE, ctypes.c_void_p(ds.data_ptr()), stream)
    assert rc == 0
    torch.cuda.synchronize()
    o, so = ora.getn(5, T.NC_INT, xr.tobytes(), T.ITYPE_DOUBLE)
    assert di.cpu().numpy()[3:3 + 8 * n].tobytes() == o.tobytes() and int(ds.item()) == so


def test_errors(torch_cuda):
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    x = np.zeros(64, np.uint8)
    assert lib.pncx_putn(5, 99, x.ctypes.data, x.ctypes.data, 4, T.ITYPE_INT, None) == T.NC_EBADTYPE
    assert lib.pncx_putn(5, T.NC_INT, x.ctypes.data, x.ctypes.data, 4, 77, None) == T.NC_EBADTYPE
    assert lib.pncx_putn(5, T.NC_CHAR, x.ctypes.data, x.ctypes.data, 4, T.ITYPE_INT, None) == T.NC_ECHAR
    assert lib.pncx_getn(5, T.NC_INT, x.ctypes.data, x.ctypes.data, 4, T.ITYPE_CHAR) == T.NC_ECHAR
    assert lib.pncx_getn(5, T.NC_INT, x.ctypes.data, x.ctypes.data, 0, T.ITYPE_INT) == T.NC_NOERR
    # NC_CHAR <-> char is a copy
    src = np.frombuffer(b"hello, netcdf!!!", np.uint8).copy()
    dst = np.zeros(16, np.uint8)
    assert lib.pncx_getn(5, T.NC_CHAR, src.ctypes.data, dst.ctypes.data, 16, T.ITYPE_CHAR) == 0
    assert dst.tobytes() == b"hello, netcdf!!!"


def test_put_leaves_user_buffer_intact(torch_cuda):
    """test_erange.c:199,217: the caller's put buffer is never altered."""
    from pnetcdf_amd import pncx
    ib = np.array([-129, 256, 5, 70000] * 1000, np.int32)
    keep = ib.copy()
    xb = np.zeros(ib.size, np.uint8)
    st = pncx.putn(5, T.NC_BYTE, xb, ib, ib.size, T.ITYPE_INT, T.fill_bytes(T.NC_BYTE))
    assert st == T.NC_ERANGE and np.array_equal(ib, keep)


# ------------------------------------------------------------------- batch
def _c4_segments(rng, nvar=256, nel=1 << 14, mixed_cast=False):
    segs = []
    for v in range(nvar):
        if v % 2 == 0:
            xt, it = T.NC_SHORT, (T.ITYPE_FLOAT if mixed_cast else T.ITYPE_SHORT)
            if mixed_cast:
                ib = rng.uniform(-40000, 40000, nel).astype(np.float32)
            else:
                ib = rng.integers(-32768, 32767, nel, dtype=np.int16)
        else:
            xt, it = T.NC_FLOAT, T.ITYPE_FLOAT
            ib = rng.standard_normal(nel).astype(np.float32)
        segs.append(dict(dir=T.PNCX_PUT, cdf_ver=5, xtype=xt, itype=it, nelems=nel,
                         xbuf=np.zeros(nel * T.xlen(xt), np.uint8), ibuf=ib, fill=T.fill_bytes(xt)))
    return segs


@pytest.mark.parametrize("mixed_cast", [False, True])
def test_host_batch_c4(torch_cuda, mixed_cast):
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(0x5EED0004)
    segs = _c4_segments(rng, nel=1 << 20, mixed_cast=mixed_cast)     # config 4's own size
    st = pncx.batch(segs)
    for s, stv in zip(segs, st):
        xb, so = ora.putn(5, s["xtype"], s["ibuf"], s["itype"], s["fill"])
        assert stv == so and s["xbuf"].tobytes() == xb


def test_dev_batch_mixed_classes(torch_cuda):
    """Segments of many classes, sizes and alignments in one call."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(11)
    segs, refs = [], []
    combos = [(T.PNCX_GET, T.NC_INT, T.ITYPE_DOUBLE), (T.PNCX_PUT, T.NC_SHORT, T.ITYPE_FLOAT),
              (T.PNCX_GET, T.NC_DOUBLE, T.ITYPE_DOUBLE), (T.PNCX_PUT, T.NC_BYTE, T.ITYPE_INT),
              (T.PNCX_GET, T.NC_UINT64, T.ITYPE_FLOAT), (T.PNCX_PUT, T.NC_USHORT, T.ITYPE_SCHAR),
              (T.PNCX_GET, T.NC_SHORT, T.ITYPE_SHORT), (T.PNCX_PUT, T.NC_FLOAT, T.ITYPE_FLOAT)]
    for k in range(40):
        d, xt, it = combos[k % len(combos)]
        n = int(rng.integers(0, 20000))
        raw = rng.integers(0, 256, n * 8 + 8, dtype=np.uint8)
        if d == T.PNCX_GET:
            xin = raw[: n * T.xlen(xt)].tobytes()
            exp, so = ora.getn(5, xt, xin, it)
            dx = torch.from_numpy(np.frombuffer(xin + b"\0" * 16, np.uint8).copy()).cuda()
            di = torch.zeros(n * T.ilen(it) + 16, dtype=torch.uint8, device="cuda")
            refs.append((di, exp.tobytes(), so, n * T.ilen(it)))
        else:
            ib = np.frombuffer(raw.tobytes(), T.ITYPE_NP[it])[:n].copy()
            xb, so = ora.putn(5, xt, ib, it, T.fill_bytes(xt))
            di = torch.from_numpy(np.frombuffer(ib.tobytes() + b"\0" * 16, np.uint8).copy()).cuda()
            dx = torch.zeros(n * T.xlen(xt) + 16, dtype=torch.uint8, device="cuda")
            refs.append((dx, xb, so, n * T.xlen(xt)))
        segs.append(dict(dir=d, cdf_ver=5, xtype=xt, itype=it, nelems=n, xbuf=dx, ibuf=di,
                         fill=T.fill_bytes(xt) if d == T.PNCX_PUT else None))
    st = pncx.dev_batch(segs)
    torch.cuda.synchronize()
    for (buf, exp, so, nb), stv in zip(refs, st):
        assert stv == so
        assert buf.cpu().numpy()[:nb].tobytes() == exp


XTYPES = [T.NC_BYTE, T.NC_UBYTE, T.NC_SHORT, T.NC_USHORT, T.NC_INT, T.NC_UINT, T.NC_FLOAT, T.NC_DOUBLE,
          T.NC_INT64, T.NC_UINT64]


@pytest.mark.parametrize("xt", XTYPES, ids=[T.XNAME[x] for x in XTYPES])
def test_dev_batch_every_external_type(torch_cuda, xt):
    """The conversion kernels are one code object per external type
    (pncx_kern_xt.c dispatches): a batch of get and put segments of this
    type with three converting internal types, each against the oracle, so
    every type's batch entry points run (the per-pair tests cover pncxk_get
    and pncxk_put)."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(0xB7 + xt)
    its = [i for i in (T.ITYPE_DOUBLE, T.ITYPE_FLOAT, T.ITYPE_INT, T.ITYPE_SCHAR) if T.XNAME[xt] != T.INAME[i]][:3]
    segs, refs = [], []
    for d in (T.PNCX_GET, T.PNCX_PUT):
        for it in its:
            n = int(rng.integers(1000, 30000))
            raw = rng.integers(0, 256, n * 8 + 8, dtype=np.uint8)
            if d == T.PNCX_GET:
                xin = raw[: n * T.xlen(xt)].tobytes()
                exp, so = ora.getn(5, xt, xin, it)
                dx = torch.from_numpy(np.frombuffer(xin + b"\0" * 16, np.uint8).copy()).cuda()
                di = torch.zeros(n * T.ilen(it) + 16, dtype=torch.uint8, device="cuda")
                refs.append((di, exp.tobytes(), so, n * T.ilen(it)))
            else:
                ib = np.frombuffer(raw.tobytes(), T.ITYPE_NP[it])[:n].copy()
                xb, so = ora.putn(5, xt, ib, it, T.fill_bytes(xt))
                di = torch.from_numpy(np.frombuffer(ib.tobytes() + b"\0" * 16, np.uint8).copy()).cuda()
                dx = torch.zeros(n * T.xlen(xt) + 16, dtype=torch.uint8, device="cuda")
                refs.append((dx, xb, so, n * T.xlen(xt)))
            segs.append(dict(dir=d, cdf_ver=5, xtype=xt, itype=it, nelems=n, xbuf=dx, ibuf=di,
                             fill=T.fill_bytes(xt) if d == T.PNCX_PUT else None))
    st = pncx.dev_batch(segs)
    torch.cuda.synchronize()
    for (buf, exp, so, nb), stv in zip(refs, st):
        assert stv == so
        assert buf.cpu().numpy()[:nb].tobytes() == exp


def test_dev_batch_plan_cache_statuses(torch_cuda):
    """A repeated segment list reuses the device plan (no upload); statuses
    carry a per-call epoch, so they follow each call's data and never report
    a stale NC_ERANGE.  Uniform, grouped (3 sizes) and mapped (12 sizes)
    classes, double -> NC_SHORT puts, outputs vs the oracle every round."""
    import ctypes
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(12)
    for sizes in ([4096] * 6, [4096, 10000, 4096, 777000, 10000, 4096], [1000 + 4099 * k for k in range(12)]):
        fill = np.frombuffer(T.fill_bytes(T.NC_SHORT) + b"\0" * 8, np.uint8).copy()
        ins = [torch.zeros(n, dtype=torch.float64, device="cuda") for n in sizes]
        outs = [torch.zeros(n * 2 + 16, dtype=torch.uint8, device="cuda") for n in sizes]
        arr = (pncx.Seg * len(sizes))(*[pncx.Seg(T.PNCX_PUT, 5, T.NC_SHORT, T.ITYPE_DOUBLE, n, outs[k].data_ptr(),
                                                 ins[k].data_ptr(), fill.ctypes.data) for k, n in enumerate(sizes)])
        st = (ctypes.c_int * len(sizes))()
        for rnd in range(4):
            bad = {k for k in range(len(sizes)) if (k + rnd) % 3 == 0}
            host = []
            for k, n in enumerate(sizes):
                v = rng.uniform(-30000, 30000, n)
                if k in bad:
                    v[int(rng.integers(0, n))] = 1e9
                ins[k].copy_(torch.from_numpy(v))
                host.append(v)
            torch.cuda.synchronize()
            pncx.lib().pncx_dev_batch(arr, len(sizes), st, None)
            torch.cuda.synchronize()
            assert list(st) == [T.NC_ERANGE if k in bad else 0 for k in range(len(sizes))], (sizes, rnd)
            for k, n in enumerate(sizes):
                exp, so = ora.putn(5, T.NC_SHORT, host[k], T.ITYPE_DOUBLE, T.fill_bytes(T.NC_SHORT))
                assert outs[k].cpu().numpy()[:n * 2].tobytes() == exp, (sizes, rnd, k)


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_dev_batch_plan_cache_fill_change(torch_cuda, mode):
    """The cached plan carries the fill value, the segment array only the
    fill's address: changing *fillp between two calls with a byte-identical
    segment array must re-plan, so the second call's ERANGE elements get the
    second fill.  Both pncx_dev_batch and
    pncx_dev_batch_async, against the oracle's putn with each fill."""
    import ctypes
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(77)
    sizes = [4096, 4096, 10000, 4096]
    fill = np.zeros(16, np.uint8)
    ins = [torch.zeros(n, dtype=torch.float64, device="cuda") for n in sizes]
    outs = [torch.zeros(n * 2 + 16, dtype=torch.uint8, device="cuda") for n in sizes]
    arr = (pncx.Seg * len(sizes))(*[pncx.Seg(T.PNCX_PUT, 5, T.NC_SHORT, T.ITYPE_DOUBLE, n, outs[k].data_ptr(),
                                             ins[k].data_ptr(), fill.ctypes.data) for k, n in enumerate(sizes)])
    st = (ctypes.c_int * len(sizes))()
    dst = torch.zeros(len(sizes), dtype=torch.int32, device="cuda")
    host = []
    for k, n in enumerate(sizes):
        v = rng.uniform(-30000, 30000, n)
        v[::7] = 1e9                                    # ERANGE every 7th element
        ins[k].copy_(torch.from_numpy(v))
        host.append(v)
    torch.cuda.synchronize()
    for fv in (-1234, 4321, -32767, 77):
        fill[:2] = np.frombuffer(np.int16(fv).tobytes(), np.uint8)   # native order, as ncmpio_inq_var_fill
        if mode == "sync":
            assert pncx.lib().pncx_dev_batch(arr, len(sizes), st, None) == T.NC_ERANGE
            assert list(st) == [T.NC_ERANGE] * len(sizes)
        else:
            dst.zero_()
            torch.cuda.synchronize()
            assert pncx.lib().pncx_dev_batch_async(arr, len(sizes), ctypes.c_void_p(dst.data_ptr()), None) == 0
            torch.cuda.synchronize()
            assert dst.cpu().tolist() == [T.NC_ERANGE] * len(sizes)
        for k, n in enumerate(sizes):
            exp, so = ora.putn(5, T.NC_SHORT, host[k], T.ITYPE_DOUBLE, bytes(fill[:2]))
            assert so == T.NC_ERANGE
            assert outs[k].cpu().numpy()[:n * 2].tobytes() == exp, (mode, fv, k)


def test_dev_batch_kernel_timing(torch_cuda):
    """pncx_dev_batch_timing: events around the batch kernels of each call
    (first call plans and uploads, the next ones hit the plan cache); the
    summed time and call count reset on enable and stop when disabled."""
    import ctypes
    torch = torch_cuda
    from pnetcdf_amd import pncx
    L = pncx.lib()
    sizes = [1 << 16, 1 << 15, 1 << 16]
    ins = [torch.arange(n, dtype=torch.float32, device="cuda") for n in sizes]
    outs = [torch.zeros(n * 4, dtype=torch.uint8, device="cuda") for n in sizes]
    arr = (pncx.Seg * 3)(*[pncx.Seg(T.PNCX_PUT, 5, T.NC_FLOAT, T.ITYPE_FLOAT, n, outs[k].data_ptr(),
                                    ins[k].data_ptr(), None) for k, n in enumerate(sizes)])
    st = (ctypes.c_int * 3)()
    tot, calls = ctypes.c_double(), ctypes.c_longlong()
    assert L.pncx_dev_batch_timing(1) == 0
    for _ in range(3):
        assert L.pncx_dev_batch(arr, 3, st, None) == 0
    assert L.pncx_dev_batch_kernel_ms(ctypes.byref(tot), ctypes.byref(calls)) == 0
    assert calls.value == 3 and 0 < tot.value < 1000
    assert L.pncx_dev_batch_timing(0) == 0
    assert L.pncx_dev_batch(arr, 3, st, None) == 0
    assert L.pncx_dev_batch_kernel_ms(ctypes.byref(tot), ctypes.byref(calls)) == 0 and calls.value == 0
    exp = np.arange(sizes[1], dtype=">f4").tobytes()
    assert outs[1].cpu().numpy().tobytes() == exp
    # async calls are timed too; more calls than the event ring holds (256)
    dst = torch.zeros(3, dtype=torch.int32, device="cuda")
    assert L.pncx_dev_batch_timing(1) == 0
    for _ in range(300):
        assert L.pncx_dev_batch_async(arr, 3, ctypes.c_void_p(dst.data_ptr()), None) == 0
    assert L.pncx_dev_batch_kernel_ms(ctypes.byref(tot), ctypes.byref(calls)) == 0
    assert calls.value == 300 and 0 < tot.value < 10000
    # two classes and a flag reduce (float -> NC_SHORT with NC_ERANGE + a swap):
    # each class kernel carries its own event pair, the reduce is not timed
    vals = torch.tensor([1.0, 4e4, -2.0, 7.0] * 4096, dtype=torch.float32, device="cuda")
    xs = torch.zeros(vals.numel() * 2, dtype=torch.uint8, device="cuda")
    fill = (ctypes.c_uint8 * 8)(0x01, 0x80)
    arr2 = (pncx.Seg * 2)(pncx.Seg(T.PNCX_PUT, 5, T.NC_SHORT, T.ITYPE_FLOAT, vals.numel(), xs.data_ptr(),
                                   vals.data_ptr(), ctypes.cast(fill, ctypes.c_void_p).value), arr[0])
    st2 = (ctypes.c_int * 2)()
    assert L.pncx_dev_batch_timing(1) == 0
    for _ in range(4):
        assert L.pncx_dev_batch(arr2, 2, st2, None) == T.NC_ERANGE
        assert list(st2) == [T.NC_ERANGE, 0]
    assert L.pncx_dev_batch_kernel_ms(ctypes.byref(tot), ctypes.byref(calls)) == 0
    assert calls.value == 4 and 0 < tot.value < 1000
    assert L.pncx_dev_batch_timing(0) == 0
    got = xs.cpu().numpy()[:8].tobytes()
    assert got == bytes([0x00, 0x01, 0x80, 0x01, 0xff, 0xfe, 0x00, 0x07])


def test_dev_batch_async(torch_cuda):
    """pncx_dev_batch_async: the same conversions as the synchronous batch,
    statuses in the caller's device words (NC_ERANGE or untouched), calls
    queued back to back on a cached plan, and sync / async calls alternating
    (each switch re-plans after waiting for the async stream).  Classes:
    double->NC_SHORT puts (ERANGE-capable), same-type swaps, and one
    NULL-fill NC_BYTE<-int put that runs outside the class kernels."""
    import ctypes
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    L = pncx.lib()
    rng = np.random.default_rng(21)
    sizes = [5000, 70001, 4096, 123457, 999, 65536]
    kinds = ["short", "short", "swap", "swap", "byte_null", "short"]
    fill = np.frombuffer(T.fill_bytes(T.NC_SHORT) + b"\0" * 8, np.uint8).copy()
    ins, outs, segs = [], [], []
    for k, (n, kind) in enumerate(zip(sizes, kinds)):
        if kind == "short":
            ins.append(torch.zeros(n, dtype=torch.float64, device="cuda"))
            outs.append(torch.zeros(n * 2 + 16, dtype=torch.uint8, device="cuda"))
            segs.append(pncx.Seg(T.PNCX_PUT, 5, T.NC_SHORT, T.ITYPE_DOUBLE, n, outs[k].data_ptr(), ins[k].data_ptr(),
                                 fill.ctypes.data))
        elif kind == "swap":
            ins.append(torch.zeros(n, dtype=torch.int32, device="cuda"))
            outs.append(torch.zeros(n * 4 + 16, dtype=torch.uint8, device="cuda"))
            segs.append(pncx.Seg(T.PNCX_PUT, 5, T.NC_INT, T.ITYPE_INT, n, outs[k].data_ptr(), ins[k].data_ptr(), None))
        else:
            ins.append(torch.zeros(n, dtype=torch.int32, device="cuda"))
            outs.append(torch.zeros(n + 16, dtype=torch.uint8, device="cuda"))
            segs.append(pncx.Seg(T.PNCX_PUT, 5, T.NC_BYTE, T.ITYPE_INT, n, outs[k].data_ptr(), ins[k].data_ptr(), None))
    arr = (pncx.Seg * len(sizes))(*segs)
    dst = torch.zeros(len(sizes), dtype=torch.int32, device="cuda")
    hst = (ctypes.c_int * len(sizes))()

    def fresh(rnd):
        host = []
        for k, (n, kind) in enumerate(zip(sizes, kinds)):
            if kind == "short":
                v = rng.uniform(-30000, 30000, n)
                if (k + rnd) % 2 == 0:
                    v[int(rng.integers(0, n))] = 1e9
            elif kind == "swap":
                v = rng.integers(-2 ** 31, 2 ** 31, n).astype(np.int32)
            else:
                v = rng.integers(-300, 300, n).astype(np.int32)
            ins[k].copy_(torch.from_numpy(v))
            outs[k].zero_()
            host.append(v)
        return host

    def check(host, statuses):
        for k, (n, kind) in enumerate(zip(sizes, kinds)):
            if kind == "short":
                exp, est = ora.putn(5, T.NC_SHORT, host[k], T.ITYPE_DOUBLE, T.fill_bytes(T.NC_SHORT))
                nb = n * 2
            elif kind == "swap":
                exp, est = ora.putn(5, T.NC_INT, host[k], T.ITYPE_INT, None)
                nb = n * 4
            else:
                exp, est = ora.putn(5, T.NC_BYTE, host[k], T.ITYPE_INT, None, xinit=b"\0" * n)
                nb = n
            assert outs[k].cpu().numpy()[:nb].tobytes() == exp, (k, kind)
            assert statuses[k] == est, (k, kind, statuses[k], est)

    for rnd in range(6):
        host = fresh(rnd)
        torch.cuda.synchronize()
        if rnd % 3 == 2:                           # synchronous call in between: its own plan
            L.pncx_dev_batch(arr, len(sizes), hst, None)
            check(host, list(hst))
        else:
            dst.zero_()
            assert L.pncx_dev_batch_async(arr, len(sizes), ctypes.c_void_p(dst.data_ptr()), None) == 0
            torch.cuda.synchronize()
            check(host, dst.cpu().tolist())
    # back to back on the cached plan: the last call's outputs and statuses
    host = fresh(1)
    torch.cuda.synchronize()
    dst.zero_()
    for _ in range(5):
        assert L.pncx_dev_batch_async(arr, len(sizes), ctypes.c_void_p(dst.data_ptr()), None) == 0
    torch.cuda.synchronize()
    check(host, dst.cpu().tolist())
    # the same plan queued on two streams in turn (the library drains the
    # first stream before the plan is used from the second)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    host = fresh(2)
    torch.cuda.synchronize()
    dst.zero_()
    for s in (sa, sb, sa):
        assert L.pncx_dev_batch_async(arr, len(sizes), ctypes.c_void_p(dst.data_ptr()),
                                      ctypes.c_void_p(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    check(host, dst.cpu().tolist())
    assert L.pncx_dev_batch_async(arr, len(sizes), None, None) == T.NC_EINVAL


def test_dev_batch_async_cached_two_streams(torch_cuda):
    """a plan that runs entirely in class kernels is cached: async calls then
    touch no host memory; queued from two streams in turn (the library drains
    the first before the plan is used from the second), then a synchronous
    call (a different plan) after them"""
    import ctypes
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    L = pncx.lib()
    rng = np.random.default_rng(22)
    sizes = [70001, 4096, 123457]
    fill = np.frombuffer(T.fill_bytes(T.NC_SHORT) + b"\0" * 8, np.uint8).copy()
    ins = [torch.zeros(n, dtype=torch.float64, device="cuda") for n in sizes]
    outs = [torch.zeros(n * 2 + 16, dtype=torch.uint8, device="cuda") for n in sizes]
    arr = (pncx.Seg * 3)(*[pncx.Seg(T.PNCX_PUT, 5, T.NC_SHORT, T.ITYPE_DOUBLE, n, outs[k].data_ptr(),
                                    ins[k].data_ptr(), fill.ctypes.data) for k, n in enumerate(sizes)])
    dst = torch.zeros(3, dtype=torch.int32, device="cuda")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for rnd in range(3):
        host = []
        for k, n in enumerate(sizes):
            v = rng.uniform(-30000, 30000, n)
            if k == rnd:
                v[n // 2] = -1e12
            ins[k].copy_(torch.from_numpy(v))
            host.append(v)
        torch.cuda.synchronize()
        dst.zero_()
        torch.cuda.synchronize()
        for s in (sa, sb, sa, sb):
            assert L.pncx_dev_batch_async(arr, 3, ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(s.cuda_stream)) == 0
        torch.cuda.synchronize()
        assert dst.cpu().tolist() == [T.NC_ERANGE if k == rnd else 0 for k in range(3)]
        for k, n in enumerate(sizes):
            exp, _ = ora.putn(5, T.NC_SHORT, host[k], T.ITYPE_DOUBLE, T.fill_bytes(T.NC_SHORT))
            assert outs[k].cpu().numpy()[:n * 2].tobytes() == exp
    st = (ctypes.c_int * 3)()
    assert L.pncx_dev_batch(arr, 3, st, None) == T.NC_ERANGE and list(st) == [0, 0, T.NC_ERANGE]


# ------------------------------------------- full-size (BASELINE) properties
def _splitmix64_torch(torch, n, seed, chunk=1 << 27):
    """splitmix64 stream on the GPU (element i = mix(seed + (i+1)*golden)),
    generated in chunks to bound temporaries; int64 arithmetic wraps."""
    out = torch.empty(n, dtype=torch.int64, device="cuda")
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        z = torch.arange(s + 1, s + 1 + m, dtype=torch.int64, device="cuda")
        z.mul_(-7046029254386353131).add_(seed)                    # 0x9E3779B97F4A7C15
        z = (z ^ ((z >> 30) & 0x3FFFFFFFF)) * -4658895280553007687  # 0xBF58476D1CE4E5B9
        z = (z ^ ((z >> 27) & 0x1FFFFFFFFF)) * -7723592293110705685 # 0x94D049BB133111EB
        out[s:s + m] = z ^ ((z >> 31) & 0x1FFFFFFFF)
    return out


def _splitmix64_np(idx, seed):
    z = (idx.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return (z ^ (z >> np.uint64(31))).view(np.int64)


def _splitmix64_chunk(torch, s, m, seed):
    """elements s..s+m-1 of the _splitmix64_torch stream"""
    z = torch.arange(s + 1, s + 1 + m, dtype=torch.int64, device="cuda")
    z.mul_(-7046029254386353131).add_(seed)
    z = (z ^ ((z >> 30) & 0x3FFFFFFFF)) * -4658895280553007687
    z = (z ^ ((z >> 27) & 0x1FFFFFFFFF)) * -7723592293110705685
    return z ^ ((z >> 31) & 0x1FFFFFFFF)


def _check_swapped_every_element(torch, x, n, seed, step=1 << 27):
    """every element of x equals the byte-reversed splitmix64 value it was
    made from (regenerated chunk by chunk on the GPU, reversed by torch)"""
    for s in range(0, n, step):
        m = min(step, n - s)
        ref = _splitmix64_chunk(torch, s, m, seed).view(torch.uint8).view(-1, 8).flip(1).reshape(-1)
        assert torch.equal(x[s:s + m].view(torch.uint8), ref), s
        del ref


def _full_size_swap(torch, gib, seed):
    from oracle import oracle as O
    from pnetcdf_amd import pncx
    n = (gib << 30) // 8
    x = _splitmix64_torch(torch, n, seed)
    pncx.dev_in_swapn(x, n, 8)
    torch.cuda.synchronize()
    _check_swapped_every_element(torch, x, n, seed)
    # the ends against the oracle too
    idx = torch.tensor([0, 1, n // 2, n - 2, n - 1], device="cuda")
    ref = _splitmix64_np(idx.cpu().numpy(), seed)
    O.in_swapn(ref, 8)
    assert np.array_equal(x[idx].cpu().numpy(), ref)
    # swapping twice is the identity
    pncx.dev_in_swapn(x, n, 8)
    torch.cuda.synchronize()
    for s in range(0, n, 1 << 27):
        m = min(1 << 27, n - s)
        assert torch.equal(x[s:s + m], _splitmix64_chunk(torch, s, m, seed)), s
    del x
    torch.cuda.empty_cache()


@pytest.mark.slow
def test_c2_full_size_swap_every_element(torch_cuda):
    """Config 2 at its BASELINE size (32 GiB NC_DOUBLE, exactly 2^23 tiles:
    the one-shot grid): every element of one in-place swap is checked, then
    a second swap restores every element."""
    _full_size_swap(torch_cuda, 32, 0x5EED0002)


@pytest.mark.slow
def test_swap_beyond_one_shot_grid(torch_cuda):
    """A 36 GiB slab is 9.4M tiles > MAX_BLOCKS = 2^23, so k_tile's lanes
    loop (grid-stride) with the inline-asm `nt sc1` streaming stores; every
    element checked."""
    _full_size_swap(torch_cuda, 36, 0x5EED0006)


@pytest.mark.slow
def test_c3_full_size_int_to_double(torch_cuda):
    """Config 3: 2^31 NC_INT (big-endian) -> double; every element equals
    the byte-reversed int32 as float64 (torch computes the reference)."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    n = 1 << 31
    xr = _splitmix64_torch(torch, n // 2, 0x5EED0003).view(torch.int32)
    dst = torch.empty(n, dtype=torch.float64, device="cuda")
    ds = torch.zeros(1, dtype=torch.int32, device="cuda")
    pncx.dev_getn(5, T.NC_INT, xr, dst, n, T.ITYPE_DOUBLE, ds)
    torch.cuda.synchronize()
    assert int(ds.item()) == 0
    step = 1 << 26
    for s in range(0, n, step):
        native = xr[s:s + step].view(torch.uint8).view(-1, 4).flip(1).reshape(-1).view(torch.int32)
        assert torch.equal(dst[s:s + step], native.to(torch.float64))


@pytest.mark.slow
def test_large_conversions_every_element(torch_cuda):
    """k_tile over 2^25 elements (32768 blocks; the one-shot grid) for a
    narrowing, a widening and a same-size conversion, every element against
    torch on the device.  Guards the store-data hazard of the inline-asm
    streaming store (round 2: a VALU reuse of the data VGPRs two
    instructions after global_store_dwordx4 corrupted 8 of 16 bytes in
    k_tile<PutOp<NC_FLOAT, double>> at random places)."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    n = 1 << 25
    g = torch.Generator(device="cuda").manual_seed(5)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")

    def be(t):                       # native tensor -> its big-endian bytes
        es = t.element_size()
        return t.contiguous().view(torch.uint8).view(-1, es).flip(1).reshape(-1)

    for rep in range(3):
        d = torch.randn(n, dtype=torch.float64, device="cuda", generator=g) * 1e3
        x = torch.empty(n * 4, dtype=torch.uint8, device="cuda")          # double -> NC_FLOAT (narrowing)
        pncx.dev_putn(5, T.NC_FLOAT, x, d, n, T.ITYPE_DOUBLE, T.fill_bytes(T.NC_FLOAT), st)
        torch.cuda.synchronize()
        assert int(st.item()) == 0 and torch.equal(x, be(d.float())), rep
        i32 = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
        xi = be(i32)
        o = torch.empty(n, dtype=torch.float64, device="cuda")            # NC_INT -> double (widening)
        pncx.dev_getn(5, T.NC_INT, xi, o, n, T.ITYPE_DOUBLE, st)
        torch.cuda.synchronize()
        assert torch.equal(o, i32.double()), rep
        f = torch.randn(n, dtype=torch.float32, device="cuda", generator=g)
        of = torch.empty(n, dtype=torch.float32, device="cuda")           # NC_FLOAT -> float (swap)
        pncx.dev_getn(5, T.NC_FLOAT, be(f), of, n, T.ITYPE_FLOAT, st)
        torch.cuda.synchronize()
        assert torch.equal(of, f), rep


def _fuzz_segments(torch, rng, ora, nseg, pairs=None, dirs=None):
    """Random segments over every (cdf, xtype, itype) pair and both directions:
    sizes 0..40000 (a few large), byte offsets 0..15 on both buffers, put
    fills that are the default, a user value or NULL (the existing external
    bytes are kept where the codec reads them); expected bytes from the oracle."""
    def dev(nbytes, off, data=b""):
        t = torch.zeros(off + nbytes + 16, dtype=torch.uint8, device="cuda")
        if data:
            t[off:off + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        return t

    segs, refs = [], []
    for _ in range(nseg):
        if pairs is None:
            cdf, xt, it, _k = PAIRS[int(rng.integers(0, len(PAIRS)))]
            d = T.PNCX_GET if rng.random() < 0.5 else T.PNCX_PUT
        else:
            j = int(rng.integers(0, len(pairs)))
            cdf, xt, it = pairs[j]
            d = dirs[j]
        n = int(rng.integers(0, 40000)) if rng.random() < 0.9 else int(rng.integers(200000, 600000))
        ox, oi = int(rng.integers(0, 16)), int(rng.integers(0, 16))
        xs, isz = T.xlen(xt), T.ilen(it)
        if rng.random() < 0.5:
            raw = rng.integers(0, 256, n * 8, dtype=np.uint8).tobytes()       # any bits
        else:                                                                 # small values: mostly in range
            raw = rng.integers(-100, 100, n).astype(np.int64).tobytes()
        fill = None
        if d == T.PNCX_GET:
            xin = raw[: n * xs]
            exp, so = ora.getn(cdf, xt, xin, it)
            dx, di = dev(n * xs, ox, xin), dev(n * isz, oi)
            refs.append((di, oi, exp.tobytes(), so, n * isz, None))
        else:
            if T.ITYPE_NP[it] in (np.float32, np.float64) and rng.random() < 0.5:
                ib = rng.uniform(-1e5, 1e5, n).astype(T.ITYPE_NP[it])
            else:
                ib = np.frombuffer(raw[: n * isz], T.ITYPE_NP[it]).copy()
            u = rng.random()
            if u < 0.4:
                fill = T.fill_bytes(xt)
            elif u < 0.8:
                fill = rng.integers(0, 256, xs, dtype=np.uint8).tobytes()
            xinit = rng.integers(0, 256, n * xs, dtype=np.uint8).tobytes()
            xb, so = ora.putn(cdf, xt, ib, it, fill, xinit=xinit if fill is None else None)
            dx, di = dev(n * xs, ox, xinit), dev(n * isz, oi, ib.tobytes())
            refs.append((dx, ox, xb, so, n * xs, xinit if fill is None else None))
        segs.append(dict(dir=d, cdf_ver=cdf, xtype=xt, itype=it, nelems=n, xbuf=dx[ox:], ibuf=di[oi:], fill=fill))
    return segs, refs


def _check_refs(refs, st):
    for k, ((buf, off, exp, so, nb, _x), stv) in enumerate(zip(refs, st)):
        assert stv == so, (k, stv, so)
        got = buf[off:off + nb].cpu().numpy().tobytes()
        assert got == exp, k


def _reset_outputs(torch, refs):
    """zero the outputs, or restore the prior external bytes a NULL fill keeps"""
    for buf, off, exp, so, nb, xinit in refs:
        buf[off:off + nb] = 0
        if xinit:
            buf[off:off + nb] = torch.frombuffer(bytearray(xinit), dtype=torch.uint8).cuda()


# (direction, xtype, itype) of the conversion class beside the same-type
# swaps: the C4 NC_ERANGE variant, a direct class, LDS narrowing and
# widening tiles, and an 8:1 class whose capped occupancy does not fuse
FUSE_CLASSES = [(T.PNCX_PUT, T.NC_SHORT, T.ITYPE_FLOAT), (T.PNCX_GET, T.NC_INT, T.ITYPE_DOUBLE),
                (T.PNCX_PUT, T.NC_FLOAT, T.ITYPE_DOUBLE), (T.PNCX_GET, T.NC_BYTE, T.ITYPE_SHORT),
                (T.PNCX_GET, T.NC_SHORT, T.ITYPE_DOUBLE), (T.PNCX_GET, T.NC_DOUBLE, T.ITYPE_SCHAR)]


@pytest.mark.parametrize("cls", FUSE_CLASSES, ids=lambda c: f"{'get' if c[0] == T.PNCX_GET else 'put'}_"
                         f"{T.XNAME[c[1]]}_{T.INAME[c[2]]}")
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("lanes", [256, 1024])
def test_dev_batch_fused_two_classes(torch_cuda, cls, seed, lanes, knob):
    """With PNCX_BATCH_FUSE=1 (off by default: no faster) a batch
    of exactly one conversion class and same-type swaps runs as ONE fused
    launch (k_batch_fused: 256-lane blocks of one conversion tile or
    a quarter swap block, or 1024-lane blocks of four tiles or one swap block;
    a class with capped occupancy falls back to two launches).  Random sizes (tile counts not multiples of four, scalar heads
    and tails), offsets, fills and NC_ERANGE: bit-exact against the oracle,
    synchronous (twice, the second from the plan cache) and asynchronous."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    knob("BATCH_FUSE", "1")
    knob("FUSE_LANES", str(lanes))
    ora = OracleConv()
    rng = np.random.default_rng(0xF05E + seed)
    d, xt, it = cls
    swaps = [(5, T.NC_FLOAT, T.ITYPE_FLOAT), (5, T.NC_SHORT, T.ITYPE_SHORT), (5, T.NC_DOUBLE, T.ITYPE_DOUBLE),
             (5, T.NC_INT, T.ITYPE_INT)]
    pairs = [(5, xt, it)] * 4 + swaps
    dirs = [d] * 4 + [T.PNCX_PUT, T.PNCX_GET, T.PNCX_PUT, T.PNCX_GET]
    segs, refs = _fuzz_segments(torch, rng, ora, 40, pairs, dirs)
    _check_refs(refs, pncx.dev_batch(segs))
    _reset_outputs(torch, refs)
    _check_refs(refs, pncx.dev_batch(segs))
    _reset_outputs(torch, refs)
    dst = torch.zeros(len(segs), dtype=torch.int32, device="cuda")
    assert pncx.dev_batch_async(segs, dst) == 0
    torch.cuda.synchronize()
    want = [r[3] for r in refs]
    assert dst.cpu().tolist() == want
    for k, (buf, off, exp, so, nb, _x) in enumerate(refs):
        assert buf[off:off + nb].cpu().numpy().tobytes() == exp, k


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_dev_batch_fuzz_all_pairs(torch_cuda, seed):
    """Random batches over all 221 pairs x both directions (misaligned, NULL /
    default / user fills), synchronous and asynchronous, each called twice
    (the second call reuses the cached plan, after the outputs are reset):
    bit-exact outputs and statuses against the oracle every time."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(0xF022 + seed)
    segs, refs = _fuzz_segments(torch, rng, ora, 90)
    _check_refs(refs, pncx.dev_batch(segs))
    _reset_outputs(torch, refs)
    _check_refs(refs, pncx.dev_batch(segs))
    # asynchronous form on fresh inputs: statuses land in device words
    segs, refs = _fuzz_segments(torch, rng, ora, 90)
    arr = (pncx.Seg * len(segs))()
    keep = []
    for k, s in enumerate(segs):
        fb = None
        if s["fill"] is not None:
            fb = np.frombuffer(bytes(s["fill"]) + b"\0" * 8, np.uint8).copy()
            keep.append(fb)
        arr[k] = pncx.Seg(s["dir"], s["cdf_ver"], s["xtype"], s["itype"], s["nelems"], s["xbuf"].data_ptr(),
                          s["ibuf"].data_ptr(), None if fb is None else fb.ctypes.data)
    dst = torch.zeros(len(segs), dtype=torch.int32, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for rep in range(2):
        if rep:
            _reset_outputs(torch, refs)
            dst.zero_()
        rc = pncx.lib().pncx_dev_batch_async(arr, len(segs), ctypes.c_void_p(dst.data_ptr()), sp)
        assert rc in (T.NC_NOERR, T.NC_ERANGE), rc
        torch.cuda.synchronize()
        _check_refs(refs, dst.cpu().tolist())


def test_flag_slots_many_streams(torch_cuda):
    """NC_ERANGE flag arrays belong to one (device, stream) and there are 32
    of them: 40 streams in turn hand slots over (the old array is retired and
    a fresh one zeroed), and a larger launch regrows a slot.  Each call's status and
    bytes must still match the oracle, with the calls of all streams queued
    before anything is read back."""
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(0x51075)
    streams = [torch.cuda.Stream() for _ in range(40)]
    fill = T.fill_bytes(T.NC_SHORT)
    checks = []
    for n in (1 << 12, 1 << 20, 1 << 14):          # small, then regrow every slot, then small again
        for k, s in enumerate(streams):
            lo, hi = (-40000.0, 40000.0) if k % 3 == 0 else (-30000.0, 30000.0)
            vals = rng.uniform(lo, hi, n).astype(np.float32)
            di = torch.from_numpy(vals).cuda()
            dx = torch.zeros(n * 2, dtype=torch.uint8, device="cuda")
            ds = torch.zeros(1, dtype=torch.int32, device="cuda")
            torch.cuda.current_stream().synchronize()        # inputs copied before the other stream reads them
            pncx.dev_putn(5, T.NC_SHORT, dx, di, n, T.ITYPE_FLOAT, fill, ds, stream=s)
            checks.append((vals, dx, ds, s))
    torch.cuda.synchronize()
    for vals, dx, ds, _s in checks:
        exp, so = ora.putn(5, T.NC_SHORT, vals, T.ITYPE_FLOAT, fill)
        assert int(ds.item()) == so
        assert dx.cpu().numpy().tobytes() == exp


def test_flag_slots_stream_per_thread(torch_cuda):
    """hipStreamPerThread is one handle for a different stream in each host
    thread, so NC_ERANGE flag arrays are keyed by the calling thread too
    (ADVICE r2): two threads putting alternately out-of-range and in-range
    values on their per-thread streams each get their own statuses."""
    import threading
    torch = torch_cuda
    from pnetcdf_amd import pncx
    ora = OracleConv()
    rng = np.random.default_rng(0x7E4D)
    fill = T.fill_bytes(T.NC_SHORT)
    n, reps = 1 << 16, 24
    work = []
    for t in range(2):
        items = []
        for k in range(reps):
            lo, hi = (-40000.0, 40000.0) if (k + t) % 2 == 0 else (-30000.0, 30000.0)
            vals = rng.uniform(lo, hi, n).astype(np.float32)
            items.append((vals, torch.from_numpy(vals).cuda(), torch.zeros(n * 2, dtype=torch.uint8, device="cuda"),
                          torch.zeros(1, dtype=torch.int32, device="cuda")))
        work.append(items)
    torch.cuda.synchronize()
    errs = []

    def run(items):
        try:
            for _vals, di, dx, ds in items:
                pncx.dev_putn(5, T.NC_SHORT, dx, di, n, T.ITYPE_FLOAT, fill, ds, stream=pncx.STREAM_PER_THREAD)
        except Exception as e:   # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(w,)) for w in work]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    assert not errs, errs
    for items in work:
        for vals, _di, dx, ds in items:
            exp, so = ora.putn(5, T.NC_SHORT, vals, T.ITYPE_FLOAT, fill)
            assert int(ds.item()) == so
            assert dx.cpu().numpy().tobytes() == exp
