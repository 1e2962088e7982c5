"""ncx.h interface (include/pncx_ncx.h) on the GPU: all 308 typed
ncmpix_{getn,pad_getn,putn,pad_putn}_<xtype>_<itype> functions against the
CPU oracle at CDF-5 semantics (the ncx layer's NC_BYTE is signed), with the
reference's pointer advance and zero padding (ncx.m4:2397-2424, 2500-2523,
2586-2615, 2709-2735), plus the text/void byte copies."""
import ctypes

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu
N = 37                                     # odd: every pad_ variant pads


@pytest.fixture(scope="module")
def ncx():
    import torch
    assert torch.cuda.is_available()
    from pnetcdf_amd import ncx as X
    X.lib()
    return X


def internal_values(rng, it, n):
    dt = np.dtype(T.ITYPE_NP[it])
    if dt.kind == "f":
        v = np.concatenate([[0.0, -0.0, 1.5, -2.5, 127.9, 128.0, -129.0, 255.5, 32767.9, 65536.0, 3e9, -3e9,
                             1e19, -1e19, np.inf, -np.inf, np.nan],
                            rng.standard_normal(n) * 10.0 ** rng.integers(0, 12, n)])[:n]
        return v.astype(dt)
    raw = np.frombuffer(rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).tobytes(), dt).copy()
    info = np.iinfo(dt)
    edges = [e for e in (0, 1, -1, int(info.min), int(info.max), 127, 128, 255, 256, 32767, 32768, 65535, 65536)
             if info.min <= e <= info.max]
    edges = np.array(edges, dtype=dt)
    raw[:len(edges)] = edges
    return raw


@pytest.mark.parametrize("with_fill", [True, False])
def test_ncx_putn_all(ncx, with_fill):
    ora = OracleConv()
    rng = np.random.default_rng(7 if with_fill else 8)
    bad = []
    for name, op, xt, it, pad in ncx.functions():
        if not op.endswith("putn"):
            continue
        vals = internal_values(rng, it, N)
        xs = T.xlen(xt)
        nb = N * xs
        padded = nb + (-nb) % 4 if pad else nb
        init = rng.integers(0, 256, padded + 8, dtype=np.uint8)
        xb = init.copy()
        fill = T.fill_bytes(xt) if with_fill else None
        fb = None if fill is None else np.frombuffer(bytes(fill) + b"\0" * 8, np.uint8).copy()
        st, adv = ncx.call_put(name, xb.ctypes.data, N, vals.ctypes.data, None if fb is None else fb.ctypes.data)
        exp, est = ora.putn(5, xt, vals, it, fill, xinit=init[:nb].tobytes())
        ok = (st == est and adv == padded and xb[:nb].tobytes() == exp and
              not xb[nb:padded].any() and xb[padded:].tobytes() == init[padded:].tobytes())
        if not ok:
            bad.append((name, st, est, adv, padded))
    assert not bad, bad[:5]


def test_ncx_getn_all(ncx):
    ora = OracleConv()
    rng = np.random.default_rng(9)
    bad = []
    for name, op, xt, it, pad in ncx.functions():
        if not op.endswith("getn"):
            continue
        xs = T.xlen(xt)
        nb = N * xs
        padded = nb + (-nb) % 4 if pad else nb
        xb = rng.integers(0, 256, padded + 8, dtype=np.uint8)
        out = np.zeros(N, T.ITYPE_NP[it])
        st, adv = ncx.call_get(name, xb.ctypes.data, N, out.ctypes.data)
        exp, est = ora.getn(5, xt, xb[:nb].tobytes(), it)
        if not (st == est and adv == padded and out.tobytes() == np.asarray(exp).tobytes()):
            bad.append((name, st, est, adv, padded))
    assert not bad, bad[:5]


@pytest.mark.parametrize("kind", ["text", "void"])
@pytest.mark.parametrize("n", [0, 1, 5, 8])
def test_ncx_text_void(ncx, kind, n):
    rng = np.random.default_rng(n)
    src = rng.integers(0, 256, n + 1, dtype=np.uint8)[:max(n, 1)]
    padded = n + (-n) % 4
    for pad in (False, True):
        nm = f"ncmpix_{'pad_' if pad else ''}putn_{kind}"
        xb = np.full(16, 0xAA, np.uint8)
        st, adv = ncx.call_put(nm, xb.ctypes.data, n, src.ctypes.data, text=True)
        want = padded if pad else n
        assert st == 0 and adv == want
        assert xb[:n].tobytes() == src[:n].tobytes() and not xb[n:want].any() and (xb[want:] == 0xAA).all()
        out = np.full(max(n, 1), 0x55, np.uint8)
        st, adv = ncx.call_get(nm.replace("putn", "getn"), xb.ctypes.data, n, out.ctypes.data)
        assert st == 0 and adv == want and out[:n].tobytes() == src[:n].tobytes()
