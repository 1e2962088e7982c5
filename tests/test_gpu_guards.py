"""Nothing outside a request: every conversion path leaves the bytes before
and after its input and output untouched.

The parity tests compare the converted range; a kernel that also stored a
few bytes past the end of its output (a last partial tile written whole)
would pass them.  In device memory such a store lands in the allocation's
slack or a neighbour's data; in a host buffer the kernel reaches through a
registration (zero copy), it lands in the user's next object or faults on
the next, unmapped page.  Here each output (and input) sits between guard
bands of a known pattern, at ragged lengths around every tile and vector
size and at offsets that move it against 16-byte alignment, through the
device launch, the device batch, the host-buffer call and the host batch;
the guards must come back intact and the values must equal the oracle's.
Host buffers are registered whole, guards included, so that such a store is
reported here rather than faulting the device (the host paths move them
with the copy engines by default since round 6; PNCX_HOST_ZC=2 runs the
zero-copy kernels over them)."""
import ctypes

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu

GUARD = 4096 + 48
PAT = 0xA5
NS = [1, 2, 3, 5, 8, 15, 16, 17, 31, 33, 63, 64, 65, 127, 129, 255, 257, 511, 513, 1023, 1025, 4095, 4097,
      65537, 262147]
# (direction, xtype, itype): swaps of every width, widening and narrowing by
# 2, 4 and 8, both directions (the direct and the LDS-staged kernel shapes)
CASES = [
    (T.PNCX_GET, T.NC_BYTE, T.ITYPE_SCHAR), (T.PNCX_GET, T.NC_SHORT, T.ITYPE_SHORT),
    (T.PNCX_GET, T.NC_INT, T.ITYPE_INT), (T.PNCX_GET, T.NC_DOUBLE, T.ITYPE_DOUBLE),
    (T.PNCX_GET, T.NC_INT, T.ITYPE_DOUBLE), (T.PNCX_GET, T.NC_SHORT, T.ITYPE_LONGLONG),
    (T.PNCX_GET, T.NC_SHORT, T.ITYPE_ULONGLONG), (T.PNCX_GET, T.NC_BYTE, T.ITYPE_DOUBLE),
    (T.PNCX_GET, T.NC_DOUBLE, T.ITYPE_SCHAR), (T.PNCX_GET, T.NC_FLOAT, T.ITYPE_SHORT),
    (T.PNCX_GET, T.NC_INT64, T.ITYPE_INT), (T.PNCX_GET, T.NC_UBYTE, T.ITYPE_FLOAT),
    (T.PNCX_PUT, T.NC_SHORT, T.ITYPE_SHORT), (T.PNCX_PUT, T.NC_DOUBLE, T.ITYPE_DOUBLE),
    (T.PNCX_PUT, T.NC_INT, T.ITYPE_DOUBLE), (T.PNCX_PUT, T.NC_FLOAT, T.ITYPE_INT),
    (T.PNCX_PUT, T.NC_SHORT, T.ITYPE_LONGLONG), (T.PNCX_PUT, T.NC_BYTE, T.ITYPE_DOUBLE),
    (T.PNCX_PUT, T.NC_DOUBLE, T.ITYPE_SCHAR), (T.PNCX_PUT, T.NC_INT64, T.ITYPE_SHORT),
    (T.PNCX_PUT, T.NC_UINT, T.ITYPE_UCHAR), (T.PNCX_PUT, T.NC_FLOAT, T.ITYPE_FLOAT),
]


def _offsets(xs, isz):
    w = max(xs, isz)
    return [o for o in (0, 1, 2, 4, 6, 8, 12) if o % w == 0 and o < 16]


def _inputs(rng, d, xt, it, n):
    """input bytes: external big-endian (get) or internal native (put), some out of range"""
    if d == T.PNCX_GET:
        xb = rng.integers(0, 256, n * T.xlen(xt), dtype=np.uint8)
        if np.dtype(T.XTYPE_NP[xt]).kind == "f":      # finite floats mostly: NaN payloads are covered elsewhere
            v = rng.uniform(-1e4, 1e4, n).astype(T.XTYPE_NP[xt])
            xb = np.frombuffer(v.astype(np.dtype(T.XTYPE_NP[xt]).newbyteorder(">")).tobytes(), np.uint8).copy()
        return xb
    dt = np.dtype(T.ITYPE_NP[it])
    if dt.kind == "f":
        v = rng.uniform(-3e5, 3e5, n).astype(dt)
    else:
        info = np.iinfo(dt)
        v = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    return np.frombuffer(v.tobytes(), np.uint8).copy()


def _expect(ora, d, xt, it, src, n):
    if d == T.PNCX_GET:
        out, st = ora.getn(5, xt, src.tobytes(), it)
        return np.frombuffer(out.tobytes(), np.uint8), st
    xb, st = ora.putn(5, xt, np.frombuffer(src.tobytes(), T.ITYPE_NP[it]), it, T.fill_bytes(xt))
    return np.frombuffer(xb, np.uint8), st


def _sizes(d, xt, it):
    xs, isz = T.xlen(xt), T.ilen(it)
    return (xs, isz) if d == T.PNCX_GET else (isz, xs)      # (source element, destination element)


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


def _check_host(buf, off, nbytes, what):
    pre, post = buf[:off], buf[off + nbytes:]
    assert (pre == PAT).all() and (post == PAT).all(), (what, "guard", int(np.nonzero(pre != PAT)[0].size),
                                                         int(np.nonzero(post != PAT)[0][:1].tolist()[0])
                                                         if (post != PAT).any() else None)


@pytest.mark.parametrize("case", CASES, ids=[f"{'get' if c[0] == T.PNCX_GET else 'put'}-x{c[1]}-i{c[2]}"
                                               for c in CASES])
def test_guards_launch_and_host(gpu, case):
    """one request per call: pncx_dev_getn/putn on HBM and pncx_getn/putn
    on host numpy buffers, every length and offset"""
    torch = gpu
    from pnetcdf_amd import pncx
    L = pncx.lib()
    ora = OracleConv()
    d, xt, it = case
    ss, ds = _sizes(d, xt, it)
    rng = np.random.default_rng(7 + xt * 16 + it)
    fb = np.frombuffer(T.fill_bytes(xt) + b"\0" * 8, np.uint8).copy()
    for n in NS:
        src = _inputs(rng, d, xt, it, n)
        exp, est = _expect(ora, d, xt, it, src, n)
        for off in _offsets(ss, ds):
            # host buffers: [guard | off | data | guard]
            hsrc = np.full(GUARD + off + n * ss + GUARD, PAT, np.uint8)
            hdst = np.full(GUARD + off + n * ds + GUARD, PAT, np.uint8)
            hsrc[GUARD + off:GUARD + off + n * ss] = src
            sp, dp = hsrc.ctypes.data + GUARD + off, hdst.ctypes.data + GUARD + off
            # registered whole, guards included: a store past the end reaches a
            # mapped guard (and is reported) instead of faulting on an unmapped page
            pncx.host_register(hsrc)
            pncx.host_register(hdst)
            try:
                if d == T.PNCX_GET:
                    rc = L.pncx_getn(5, xt, ctypes.c_void_p(sp), ctypes.c_void_p(dp), n, it)
                else:
                    rc = L.pncx_putn(5, xt, ctypes.c_void_p(dp), ctypes.c_void_p(sp), n, it,
                                     ctypes.c_void_p(fb.ctypes.data))
            finally:
                pncx.host_unregister(hsrc)
                pncx.host_unregister(hdst)
            what = ("host", case, n, off)
            assert rc == est, (what, rc, est)
            _check_host(hdst, GUARD + off, n * ds, what)
            _check_host(hsrc, GUARD + off, n * ss, what)
            assert hdst[GUARD + off:GUARD + off + n * ds].tobytes() == exp.tobytes(), what
            # device buffers, the same layout
            tsrc = torch.from_numpy(hsrc).cuda()
            tdst = torch.full((hdst.size,), PAT, dtype=torch.uint8, device="cuda")
            st = torch.zeros(1, dtype=torch.int32, device="cuda")
            s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            sp, dp = tsrc.data_ptr() + GUARD + off, tdst.data_ptr() + GUARD + off
            if d == T.PNCX_GET:
                rc = L.pncx_dev_getn(5, xt, ctypes.c_void_p(sp), ctypes.c_void_p(dp), n, it,
                                     ctypes.c_void_p(st.data_ptr()), s)
            else:
                rc = L.pncx_dev_putn(5, xt, ctypes.c_void_p(dp), ctypes.c_void_p(sp), n, it,
                                     ctypes.c_void_p(fb.ctypes.data), ctypes.c_void_p(st.data_ptr()), s)
            assert rc == 0, rc
            got = tdst.cpu().numpy()
            what = ("device", case, n, off)
            assert int(st.item()) == est, (what, int(st.item()), est)
            _check_host(got, GUARD + off, n * ds, what)
            assert got[GUARD + off:GUARD + off + n * ds].tobytes() == exp.tobytes(), what


@pytest.mark.parametrize("where", ["device", "host"])
def test_guards_batch(gpu, where):
    """many requests per call (pncx_dev_batch / pncx_batch): every case at
    several lengths and offsets, each segment between guards in one pair of
    buffers, in batches of mixed classes"""
    torch = gpu
    from pnetcdf_amd import pncx
    L = pncx.lib()
    ora = OracleConv()
    rng = np.random.default_rng(0x6A4D)
    items = []
    for case in CASES:
        d, xt, it = case
        ss, ds = _sizes(d, xt, it)
        for n in rng.choice(NS, 6, replace=False):
            offs = _offsets(ss, ds)
            items.append((case, int(n), int(offs[int(rng.integers(0, len(offs)))])))
    rng.shuffle(items)
    for b0 in range(0, len(items), 24):
        batch = items[b0:b0 + 24]
        # lay every segment out in one source and one destination buffer
        spos, dpos, stot, dtot, srcs, exps = [], [], 0, 0, [], []
        for (d, xt, it), n, off in batch:
            ss, ds = _sizes(d, xt, it)
            stot += GUARD + 16 - (stot + GUARD) % 16 + off
            spos.append(stot)
            stot += n * ss
            dtot += GUARD + 16 - (dtot + GUARD) % 16 + off
            dpos.append(dtot)
            dtot += n * ds
            src = _inputs(rng, d, xt, it, n)
            srcs.append(src)
            exps.append(_expect(ora, d, xt, it, src, n))
        hsrc = np.full(stot + GUARD, PAT, np.uint8)
        hdst = np.full(dtot + GUARD, PAT, np.uint8)
        for k, ((d, xt, it), n, off) in enumerate(batch):
            hsrc[spos[k]:spos[k] + srcs[k].size] = srcs[k]
        if where == "device":
            tsrc = torch.from_numpy(hsrc).cuda()
            tdst = torch.from_numpy(hdst).cuda()
            sb, db = tsrc.data_ptr(), tdst.data_ptr()
        else:
            sb, db = hsrc.ctypes.data, hdst.ctypes.data
        arr = (pncx.Seg * len(batch))()
        keep = []
        for k, ((d, xt, it), n, off) in enumerate(batch):
            fb = np.frombuffer(T.fill_bytes(xt) + b"\0" * 8, np.uint8).copy()
            keep.append(fb)
            xb, ib = (sb + spos[k], db + dpos[k]) if d == T.PNCX_GET else (db + dpos[k], sb + spos[k])
            arr[k] = pncx.Seg(d, 5, xt, it, n, xb, ib, None if d == T.PNCX_GET else fb.ctypes.data)
        st = (ctypes.c_int * len(batch))()
        if where == "device":
            rc = L.pncx_dev_batch(arr, len(batch), st, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            got, gsrc = tdst.cpu().numpy(), tsrc.cpu().numpy()
        else:
            pncx.host_register(hsrc)                # guards mapped too (see above)
            pncx.host_register(hdst)
            try:
                rc = L.pncx_batch(arr, len(batch), st)
            finally:
                pncx.host_unregister(hsrc)
                pncx.host_unregister(hdst)
            got, gsrc = hdst, hsrc
        assert rc in (0, T.NC_ERANGE), rc
        mask = np.zeros(got.size, bool)
        smask = np.zeros(gsrc.size, bool)
        for k, ((d, xt, it), n, off) in enumerate(batch):
            ss, ds = _sizes(d, xt, it)
            exp, est = exps[k]
            what = (where, (d, xt, it), n, off)
            assert st[k] == est, (what, st[k], est)
            assert got[dpos[k]:dpos[k] + n * ds].tobytes() == exp.tobytes(), what
            mask[dpos[k]:dpos[k] + n * ds] = True
            smask[spos[k]:spos[k] + n * ss] = True
        bad = np.nonzero(~mask & (got != PAT))[0]
        assert bad.size == 0, (where, "destination guard touched at", int(bad[0]))
        assert (gsrc[~smask] == PAT).all(), (where, "source guard touched")
