"""Fill path (fill_var_buf, ncmpio_fill.c:89-140) on the GPU.

Expected bytes: the default fill value of each xtype (pnetcdf.h.in:104-114)
encoded big-endian, which is what the reference's FILL_<X> byte tables
(ncmpio_fill.c:50-60) hold, or a user _FillValue's external bytes.
"""
import ctypes

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T

pytestmark = pytest.mark.gpu
XTS = [T.NC_CHAR] + T.NUMERIC_XTYPES


def pattern(xt, value=None):
    v = T.XTYPE_FILL[xt] if value is None else value
    return np.array([v], dtype=T.XTYPE_BE[xt]).tobytes()


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.mark.parametrize("xt", XTS, ids=[T.XNAME[x] for x in XTS])
@pytest.mark.parametrize("n", [0, 1, 7, 4099, 1 << 20])
def test_host_fill_default_and_user(torch_cuda, xt, n):
    from pnetcdf_amd import pncx
    xs = T.xlen(xt)
    buf = np.full(n * xs + 3, 0x5A, np.uint8)
    pncx.fill(xt, buf, n) if n else None
    assert buf[:n * xs].tobytes() == pattern(xt) * n
    assert buf[n * xs:].tobytes() == b"\x5a" * 3          # nothing past the end
    if xt != T.NC_CHAR:
        user = pattern(xt, 99)
        pncx.fill(xt, buf, n, user)
        assert buf[:n * xs].tobytes() == user * n


@pytest.mark.parametrize("xt", [T.NC_SHORT, T.NC_DOUBLE, T.NC_BYTE, T.NC_INT])
@pytest.mark.parametrize("offset", [0, 1, 2, 8, 12])
def test_dev_fill_offsets(torch_cuda, xt, offset):
    torch = torch_cuda
    from pnetcdf_amd import pncx
    xs = T.xlen(xt)
    n = 10007
    d = torch.full(((n + 16) * xs + 64,), 0x33, dtype=torch.uint8, device="cuda")
    lib = pncx.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.pncx_dev_fill(xt, ctypes.c_void_p(d.data_ptr() + offset * xs), n, None, sp) == 0
    torch.cuda.synchronize()
    h = d.cpu().numpy().tobytes()
    assert h[:offset * xs] == b"\x33" * (offset * xs)
    assert h[offset * xs:(offset + n) * xs] == pattern(xt) * n
    assert set(h[(offset + n) * xs:]) == {0x33}


def test_dev_fill_large_sampled(torch_cuda):
    torch = torch_cuda
    from pnetcdf_amd import pncx
    n = (3 << 30) // 8
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    pncx.dev_fill(T.NC_DOUBLE, d, n)
    torch.cuda.synchronize()
    expect = np.frombuffer(pattern(T.NC_DOUBLE), np.int64)[0]
    assert bool((d[::997] == int(expect)).all().item()) and int(d[-1].item()) == int(expect)


def test_fill_bad_type(torch_cuda):
    from pnetcdf_amd import pncx
    assert pncx.lib().pncx_fill(42, None, 10, None) == T.NC_EBADTYPE
