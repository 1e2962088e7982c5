"""First-touch record appends (round 5): the reference's own
benchmark pattern (benchmarks/C/pnetcdf_put_vara.c:193-209) writes every
record of a record variable once, past the end of the file.  On tmpfs the
library now allocates an appended range while the GPU converts
(grow_for_put), reads an inline get's chunks on several pool threads
(pio_read_split) and brings small device-buffer puts back in event-marked
pieces (put_dev_small).  None of that may change a byte: every file here is
checked against the oracle's putn, with the changes on and off, and the
file's size and numrecs against what pwrite alone would leave."""
import os
import shutil

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N
from tests import capi, cdfparse
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu

SHM = "/dev/shm"


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    return torch


@pytest.fixture
def shm_dir():
    if not os.path.isdir(SHM):
        pytest.skip("no /dev/shm")
    d = os.path.join(SHM, f"pncx_ft_{os.getpid()}")
    os.makedirs(d, exist_ok=True)
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _json(r):
    import json
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


@pytest.mark.parametrize("dev", [0, 1], ids=["host", "device"])
@pytest.mark.parametrize("threads", ["1", "8"])
def test_c1first_records_hold_the_oracle_bytes(gpu, shm_dir, dev, threads):
    """api_check c1first (bench.py's first_touch leg) at a small size: every
    appended record equals the oracle's putn of the values the program wrote
    (record r holds v + r + 1), numrecs is the record count and the file
    ends at the last record, as the reference's pwrites leave it."""
    n, nrec = (1 << 18) + 3, 6                      # an odd record size: unaligned record starts
    nc = os.path.join(shm_dir, f"c1f_{dev}_{threads}.nc")
    env = dict(os.environ, PNCX_IO_THREADS=threads)
    out = _json(capi.run([capi.exe("api_check"), "c1first", nc, str(n), str(nrec), str(dev)], env=env))
    assert out["errors"] == 0
    raw = open(nc, "rb").read()
    h = cdfparse.parse_cdf(raw)
    assert h["numrecs"] == nrec
    v = h["vars"][0]
    assert len(raw) == v["begin"] + nrec * 4 * n
    base = (np.arange(n, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32)
    ora = OracleConv()
    for r in range(nrec):
        vals = (base + np.uint32(r + 1)).view(np.int32)
        exp, st = ora.putn(5, T.NC_INT, vals, T.ITYPE_INT, T.fill_bytes(T.NC_INT))
        off = v["begin"] + r * 4 * n
        assert st == 0 and raw[off:off + 4 * n] == exp, f"record {r}"


PAIRS = [(T.NC_INT, T.ITYPE_INT), (T.NC_SHORT, T.ITYPE_FLOAT), (T.NC_DOUBLE, T.ITYPE_DOUBLE),
         (T.NC_FLOAT, T.ITYPE_DOUBLE)]


def _appends(gpu, path, xt, it, n, where, order):
    """records appended in `order` (holes when it skips), then read back"""
    torch = gpu
    rng = np.random.default_rng(0xF7 + xt * 16 + it)
    err, ncid = N.create(path, N.NC_64BIT_DATA)
    assert err == 0
    N.def_dim(ncid, "t", N.NC_UNLIMITED)
    N.def_dim(ncid, "x", n)
    N.def_var(ncid, "r", xt, [0, 1])
    assert N.enddef(ncid) == 0
    out = []
    for r in order:
        # floats reach past NC_SHORT's range (NC_ERANGE + fill); ints stay in range
        b = (rng.standard_normal(n) * (1e5 if it == T.ITYPE_FLOAT else 1e6)).astype(T.ITYPE_NP[it])
        if where == "dev":
            st = N.put_var_dev(ncid, 0, torch.from_numpy(b).cuda(), [r, 0], [1, n])
        else:
            st = N.put_var(ncid, 0, b, [r, 0], [1, n], itype=it)
        out.append(("put", r, st, b.tobytes()))
    for r in sorted(order):
        o = np.zeros(n, T.ITYPE_NP[it])
        st = N.get_var(ncid, 0, o, [r, 0], [1, n], itype=it)
        out.append(("get", r, st, o.tobytes()))
    assert N.close(ncid) == 0
    return open(path, "rb").read(), out


@pytest.mark.parametrize("where", ["host", "dev"])
@pytest.mark.parametrize("xt,it", PAIRS, ids=[f"{T.XNAME[x]}-{T.INAME[i]}" for x, i in PAIRS])
def test_appends_same_with_and_without_first_touch_paths(gpu, shm_dir, knob, xt, it, where):
    """records appended in order and with holes (3, 0, 5, 1): the same file
    bytes, statuses (NC_ERANGE included) and read-back values with the
    appended-range allocation and split reads off and on, equal to the
    oracle; the file's size is the last record's end"""
    n = (1 << 18) + 7
    order = [3, 0, 5, 1]
    runs = {}
    for mode in (0, 1):
        knob("GROW", mode)
        knob("READ_SPLIT", 4 if mode else 0)
        runs[mode] = _appends(gpu, os.path.join(shm_dir, f"a{mode}.nc"), xt, it, n, where, order)
    assert runs[0][0] == runs[1][0], "file bytes differ"
    assert runs[0][1] == runs[1][1], "statuses or read-back values differ"
    raw, out = runs[1]
    h = cdfparse.parse_cdf(raw)
    v = h["vars"][0]
    xs = T.xlen(xt)
    assert h["numrecs"] == 6 and len(raw) == v["begin"] + 6 * xs * n
    ora = OracleConv()
    for kind, r, st, b in out:
        if kind != "put":
            continue
        exp, est = ora.putn(5, xt, np.frombuffer(b, T.ITYPE_NP[it]), it, T.fill_bytes(xt))
        off = v["begin"] + r * xs * n
        assert raw[off:off + xs * n] == exp and st == est, f"record {r}"
    for r in (2, 4):                                 # never written: the holes read as zeros
        off = v["begin"] + r * xs * n
        assert raw[off:off + xs * n] == b"\0" * (xs * n)


@pytest.mark.parametrize("where", ["host", "dev"])
def test_failed_append_cuts_the_file_back(gpu, shm_dir, knob, where):
    """an appending put that grows the file (grow_for_put) and then fails
    before writing anything (PNCX_FAULT=1, test-only injection right after
    the grow) leaves the file at its size before the put -- what the
    reference's convert-then-pwrite leaves (ncmpio_getput.m4:186-214) --
    and the next put appends normally"""
    torch = gpu
    # the device put grows the file only on its one-slot path (the record
    # within one staging slot, PNCX_STAGE_MB, and at least 1 MiB)
    slot_mb = int(os.environ.get("PNCX_STAGE_MB", "32") or 32)
    n = (1 << 18) + 7 if slot_mb > 1 or slot_mb <= 0 else 1 << 18
    path = os.path.join(shm_dir, "fault.nc")
    err, ncid = N.create(path, N.NC_64BIT_DATA)
    assert err == 0
    N.def_dim(ncid, "t", N.NC_UNLIMITED)
    N.def_dim(ncid, "x", n)
    N.def_var(ncid, "r", T.NC_INT, [0, 1])
    assert N.enddef(ncid) == 0
    vals = np.arange(n, dtype=np.int32) * 3 - 7

    def put(r):
        if where == "dev":
            return N.put_var_dev(ncid, 0, torch.from_numpy(vals + r).cuda(), [r, 0], [1, n])
        return N.put_var(ncid, 0, vals + r, [r, 0], [1, n], itype=T.ITYPE_INT)

    knob("GROW", 1)                             # whatever the suite runs with
    assert put(0) == 0
    size0 = os.path.getsize(path)
    knob("FAULT", 1)
    assert put(1) == N.NC_EWRITE
    assert os.path.getsize(path) == size0, "the failed put left a grown tail"
    knob("FAULT", 0)
    assert put(1) == 0
    assert N.close(ncid) == 0
    raw = open(path, "rb").read()
    h = cdfparse.parse_cdf(raw)
    v = h["vars"][0]
    assert h["numrecs"] == 2 and len(raw) == v["begin"] + 2 * 4 * n
    ora = OracleConv()
    for r in (0, 1):
        exp, st = ora.putn(5, T.NC_INT, vals + r, T.ITYPE_INT, T.fill_bytes(T.NC_INT))
        assert raw[v["begin"] + r * 4 * n:v["begin"] + (r + 1) * 4 * n] == exp, r
