"""C programs on the reference's C interfaces, linked with this build (GPU).

  - ncmpii_check (tests/mpi/ncmpii_check.c) calls ncmpii_putn_NC_<X>,
    ncmpii_getn_NC_<X> and ncmpii_in_swapn of libpncx_ncmpii.so with real
    MPI_Datatype handles -- all 11 conversion types including MPI_LONG, and
    types with no conversion itype (NC_EBADTYPE, convert_swap.m4:245,311) --
    and every output is compared with the CPU oracle, bit for bit.
  - api_check (tests/mpi/api_check.c) is written against include/pnetcdf.h
    and linked with libpnetcdf.so (dispatcher + struct PNC_driver of the
    MI355X driver): BASELINE config 1 (1-D 2^20 NC_INT put_vara_int_all +
    get_vara_int_all, and config 3's get_vara_double_all), the
    benchmarks/C/pnetcdf_put_vara.c pattern (iput_vara_float x N +
    wait_all; blocking collective and independent) on 1, 2 and 4 ranks,
    config 4 (256 iput_vara_short/float + one wait_all, and the NC_ERANGE
    variant), and config 5's record slabs on 2 and 3 ranks.  File bytes are
    checked against the oracle's putn.
  - the reference's own benchmarks/C/pnetcdf_put_vara.c, compiled from the
    reference tree against include/pnetcdf.h (oracle/Makefile target
    ref-bench -> oracle/_ref/, built where the reference tree exists), runs
    unchanged on libpnetcdf.so.
"""
import json
import os

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from tests import capi, cdfparse
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "edge_vectors.npz"))


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"


def _ncmpii_cases(rng):
    """(case bytes, expected (status, bytes)) for putn/getn of every xtype x
    MPI type, random bits and the golden edge inputs"""
    ora = OracleConv()
    cases, exp = [], []
    for xt in T.NUMERIC_XTYPES:
        xs = T.xlen(xt)
        for cdf in ((2, 5) if xt == T.NC_BYTE else (5,)):
            for mi in list(range(11)) + list(capi.MPI_UNKNOWN):
                isz = capi.MPI_SIZE[mi]
                it = capi.MPI_IDX_ITYPE.get(mi, 0)
                k = f"{T.XNAME[xt]}_{T.INAME[it]}" if it else None
                for src in ("random", "edge"):
                    if src == "edge" and it == 0:
                        continue
                    if src == "edge":
                        ib = GOLD[f"put_{k}_in"].tobytes()
                        xb = GOLD[f"get_{k}_in"].tobytes()
                        n = len(ib) // isz
                        xb = xb[:len(xb) // xs * xs]
                        nx = len(xb) // xs
                    else:
                        n = nx = 1031
                        ib = rng.integers(0, 256, n * isz, dtype=np.uint8).tobytes()
                        xb = rng.integers(0, 256, nx * xs, dtype=np.uint8).tobytes()
                    xinit = rng.integers(0, 256, n * xs, dtype=np.uint8).tobytes()
                    for fill in (T.fill_bytes(xt), T.fill_bytes(xt, 99), None):
                        cases.append(capi.case(0, cdf, xt, mi, n, fill, ib + xinit))
                        if it == 0:
                            exp.append((T.NC_EBADTYPE, xinit))
                        else:
                            arr = np.frombuffer(ib, T.ITYPE_NP[it])
                            xo, st = ora.putn(cdf, xt, arr, it, fill, xinit=xinit)
                            exp.append((st, xo))
                    cases.append(capi.case(1, cdf, xt, mi, nx, None, xb))
                    if it == 0:
                        exp.append((T.NC_EBADTYPE, b"\0" * (nx * isz)))
                    else:
                        go, st = ora.getn(cdf, xt, xb, it)
                        exp.append((st, go.tobytes()))
    return cases, exp


def test_ncmpii_putn_getn_with_mpi_datatypes(gpu, tmp_path):
    cases, exp = _ncmpii_cases(np.random.default_rng(0x5EED00C1))
    cp, op = str(tmp_path / "c.bin"), str(tmp_path / "o.bin")
    open(cp, "wb").write(b"".join(cases))
    capi.run([capi.exe("ncmpii_check"), "run", cp, op])
    got = capi.read_results(op)
    assert len(got) == len(exp)
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not bad, (len(bad), bad[:10], got[bad[0]][0], exp[bad[0]][0])


def test_ncmpii_in_swapn(gpu, tmp_path):
    from oracle import oracle as O
    rng = np.random.default_rng(7)
    cases, exp = [], []
    for esize in (2, 3, 4, 8, 16):
        for n in (0, 1, 17, 4099, (1 << 20) + 3):
            b = rng.integers(0, 256, n * esize, dtype=np.uint8)
            r = b.copy()
            O.in_swapn(r, esize)
            cases.append(capi.case(2, 5, esize, 0, n, None, b.tobytes()))
            exp.append((0, r.tobytes()))
    cp, op = str(tmp_path / "c.bin"), str(tmp_path / "o.bin")
    open(cp, "wb").write(b"".join(cases))
    capi.run([capi.exe("ncmpii_check"), "run", cp, op])
    assert capi.read_results(op) == exp


def _json(r):
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


def _var_bytes(raw, h, name, rec=None):
    v = next(v for v in h["vars"] if v["name"] == name)
    off, per = v["extents"][rec if rec is not None else 0]
    return raw[off:off + per * T.xlen(v["xtype"])]


@pytest.mark.parametrize("dev", [0, 1], ids=["host", "device"])
def test_config1_put_get_vara_int_all(gpu, tmp_path, dev):
    """BASELINE config 1 through the public API: 2^20 NC_INT
    put_vara_int_all, then get_vara_int_all and get_vara_double_all (config
    3's read).  dev = 1: the user buffers are hipMalloc'ed, so the same
    ncmpi_* calls take the device-resident path (converted in HBM, the
    external bytes across PCIe once)."""
    n = 1 << 20
    v = np.random.default_rng(0x5EED0001).integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype(np.int32)
    v[:4] = [-2**31, 2**31 - 1, 0, -1]
    inp, nc = str(tmp_path / "in.bin"), str(tmp_path / "c1.nc")
    v.tofile(inp)
    out = _json(capi.run([capi.exe("api_check"), "c1", nc, inp, str(n), str(dev)]))
    assert out["errors"] == 0 and out["put_size"] == 4 * n and out["get_size"] == 8 * n
    raw = open(nc, "rb").read()
    h = cdfparse.parse_cdf(raw)
    exp, st = OracleConv().putn(5, T.NC_INT, v, T.ITYPE_INT, T.fill_bytes(T.NC_INT))
    assert st == 0 and _var_bytes(raw, h, "v") == exp


def _check_putvara(nc, out, nvars, length, ntimes):
    raw = open(nc, "rb").read()
    h = cdfparse.parse_cdf(raw)
    py, px, nprocs = out["py"], out["px"], out["nprocs"]
    assert h["numrecs"] == ntimes and [d[1] for d in h["dims"]] == [0, py * length, px * length]
    ora = OracleConv()
    fill = T.fill_bytes(T.NC_FLOAT)
    for i in range(nvars):
        v = next(v for v in h["vars"] if v["name"] == f"var_{i}")
        assert set(v["atts"]) == {"str_att", "float_att", "short_att"}
        for t in range(ntimes):
            off, per = v["extents"][t]
            rec = np.frombuffer(raw[off:off + per * 4], ">f4").reshape(py * length, px * length)
            for r in range(nprocs):
                by, bx = r // px, r % px
                blk = (r + i * length + np.arange(length * length)).astype(np.float32)
                exp, st = ora.putn(5, T.NC_FLOAT, blk, T.ITYPE_FLOAT, fill)
                got = rec[by * length:(by + 1) * length, bx * length:(bx + 1) * length].astype(">f4").tobytes()
                assert st == 0 and got == exp, (i, t, r)


@pytest.mark.parametrize("mode", [("1", "0"), ("0", "0"), ("0", "1"), ("1", "1")],
                         ids=["iput_wait_all", "put_all", "put_indep", "iput_wait_indep"])
def test_put_vara_benchmark_pattern_one_rank(gpu, tmp_path, mode):
    nb, indep = mode
    nc = str(tmp_path / "pv.nc")
    out = _json(capi.run([capi.exe("api_check"), "putvara", nc, "4", "64", "3", nb, indep]))
    assert out["errors"] == 0 and out["nprocs"] == 1
    _check_putvara(nc, out, 4, 64, 3)


@pytest.mark.skipif(not capi.have_mpiexec(), reason="mpiexec not available")
@pytest.mark.parametrize("nprocs", [2, 4])
def test_put_vara_benchmark_pattern_ranks(gpu, tmp_path, nprocs):
    """pnetcdf_put_vara.c's pattern on N ranks sharing one file: rank 0
    writes the header, every rank its 2-D block of every record."""
    nc = str(tmp_path / "pvn.nc")
    out = _json(capi.run([capi.exe("api_check"), "putvara", nc, "3", "48", "2", "1"], nprocs=nprocs))
    assert out["errors"] == 0 and out["nprocs"] == nprocs
    _check_putvara(nc, out, 3, 48, 2)


@pytest.mark.parametrize("dev", [0, 1], ids=["host", "device"])
@pytest.mark.parametrize("erange", [0, 1])
def test_config4_iput_batch(gpu, tmp_path, erange, dev):
    """BASELINE config 4 through the public API: 256 iput_vara_short/float
    + one wait_all (one batched conversion); erange = 1: the NC_SHORT
    variables from float in [-40000, 40000] (SURVEY §8(d) secondary).
    dev = 1: the 256 user buffers are hipMalloc'ed; the wait converts them
    with pncx_dev_batch in HBM."""
    nel = 1 << 16
    rng = np.random.default_rng(0x5EED0004)
    sh = rng.integers(-32768, 32767, 128 * nel, dtype=np.int16)
    fl = (rng.uniform(-40000, 40000, 128 * nel) if erange else rng.standard_normal(128 * nel)).astype(np.float32)
    sp, fp, nc = str(tmp_path / "s.bin"), str(tmp_path / "f.bin"), str(tmp_path / "c4.nc")
    sh.tofile(sp)
    fl.tofile(fp)
    out = _json(capi.run([capi.exe("api_check"), "c4", nc, sp, fp, str(nel), str(erange), str(dev)]))
    assert out["errors"] == 0 and out["reqs_after"] == -1          # NC_REQ_NULL after the wait
    ora = OracleConv()
    raw = open(nc, "rb").read()
    h = cdfparse.parse_cdf(raw)
    st_exp = []
    for v in range(256):
        k = v // 2
        if v % 2 == 0:
            src, it = (fl[k * nel:(k + 1) * nel], T.ITYPE_FLOAT) if erange else (sh[k * nel:(k + 1) * nel],
                                                                                T.ITYPE_SHORT)
            xt = T.NC_SHORT
        else:
            src, it, xt = fl[k * nel:(k + 1) * nel], T.ITYPE_FLOAT, T.NC_FLOAT
        exp, st = ora.putn(5, xt, src, it, T.fill_bytes(xt))
        st_exp.append(st)
        assert _var_bytes(raw, h, f"v{v}") == exp, v
    assert out["statuses"] == st_exp
    assert out["wait"] == (T.NC_ERANGE if erange else 0)
    assert (T.NC_ERANGE in st_exp) == bool(erange)


@pytest.mark.skipif(not capi.have_mpiexec(), reason="mpiexec not available")
@pytest.mark.parametrize("nprocs", [2, 3])
def test_config5_record_slabs_ranks(gpu, tmp_path, nprocs):
    """Config 5 at file level: a record variable written as record slabs,
    one per rank, with put_vara_double_all; numrecs agreed by MAX (rank 0
    holds the last records yet every rank sees all of them), then every
    rank reads every record back."""
    nrec, x = 7, 4096
    nc = str(tmp_path / "rec.nc")
    out = _json(capi.run([capi.exe("api_check"), "records", nc, str(nrec), str(x)], nprocs=nprocs))
    assert out["errors"] == 0
    raw = open(nc, "rb").read()
    h = cdfparse.parse_cdf(raw)
    assert h["numrecs"] == nrec
    ora = OracleConv()
    for r in range(nrec):
        vals = r * 1000.0 + np.arange(x) + 0.25
        exp, _ = ora.putn(5, T.NC_DOUBLE, vals, T.ITYPE_DOUBLE, T.fill_bytes(T.NC_DOUBLE))
        assert _var_bytes(raw, h, "v", r) == exp, r


REF_BENCH = os.path.join(capi.ROOT, "oracle", "_ref", "pnetcdf_put_vara")


@pytest.mark.skipif(not os.path.exists(REF_BENCH), reason="oracle/_ref/pnetcdf_put_vara not built")
@pytest.mark.parametrize("args", [["-i"], []], ids=["nonblocking", "blocking"])
def test_reference_benchmark_runs_on_libpnetcdf(gpu, tmp_path, args):
    """The reference's benchmarks/C/pnetcdf_put_vara.c, unchanged, on this
    library: exit status 0 and the file holds its values."""
    nc = str(tmp_path / "ref.nc")
    r = capi.run([REF_BENCH, "-k", "5", "-l", "32", "-n", "3", "-t", "2"] + args + [nc])
    assert "Write bandwidth" in r.stdout
    _check_putvara(nc, {"py": 1, "px": 1, "nprocs": 1}, 3, 32, 2)


@pytest.mark.parametrize("dev", [0, 1], ids=["host", "device"])
def test_config1_bench_mode(gpu, tmp_path, dev):
    """bench.py's c1 leg: repeated put_vara_int_all / get_vara_int_all on
    one open file, host or hipMalloc'ed buffers; the last get must equal
    the put and the file must hold the oracle's bytes."""
    n = 1 << 16
    nc = str(tmp_path / "c1b.nc")
    out = _json(capi.run([capi.exe("api_check"), "c1bench", nc, str(n), "3", str(dev)]))
    assert out["errors"] == 0 and out["put_ms_median"] > 0 and out["get_ms_median"] > 0
    vals = (np.arange(n, dtype=np.uint64) * 2654435761 % (1 << 32)).astype(np.uint32).view(np.int32)
    exp, st = OracleConv().putn(5, T.NC_INT, vals, T.ITYPE_INT, T.fill_bytes(T.NC_INT))
    raw = open(nc, "rb").read()
    assert st == 0 and raw[out["var_offset"]:out["var_offset"] + 4 * n] == exp


@pytest.mark.parametrize("nprocs", [1, 2])
def test_numrecs_written_by_collective_record_puts(gpu, tmp_path, nprocs):
    """ncmpio_getput.m4:272-311: a collective put of a record variable
    writes the MAX record count into the file at once; a fixed-size put
    leaves it alone.  Rank 0 reads the header bytes between the puts."""
    if nprocs > 1 and not capi.have_mpiexec():
        pytest.skip("mpiexec not available")
    nc = str(tmp_path / "nr.nc")
    out = _json(capi.run([capi.exe("api_check"), "numrecs", nc], nprocs=nprocs))
    assert out["errors"] == 0
    assert out["after_rec_put"] == nprocs
    assert out["after_fix_put"] == nprocs
    assert out["after_second_rec_put"] == nprocs + 2
    assert out["at_close"] == nprocs + 2


@pytest.mark.skipif(not capi.have_mpiexec(), reason="mpiexec not available")
def test_failed_open_and_create_keep_other_file(gpu, tmp_path):
    """an open or create that fails on one rank only fails on
    every rank, must not close the file the ranks already have open (it is
    pncx_nc id 0 on every rank), and a failed create removes its file."""
    out = _json(capi.run([capi.exe("api_check"), "openfail", str(tmp_path)], nprocs=2))
    assert out["errors"] == 0
    assert out["open"] < 0                 # NC_ENOENT on the last rank, the MIN on every rank
    assert out["create"] < 0 and out["c_exists"] == 0


def test_bput_short_bufcount(gpu, tmp_path):
    """bput_vara with a predefined buftype and bufcount short of
    the request is NC_EIOMISMATCH, not a read past the buffer."""
    out = _json(capi.run([capi.exe("api_check"), "bputshort", str(tmp_path / "b.nc")]))
    assert out["errors"] == 0 and out["short"] == T.NC_EIOMISMATCH and out["exact"] == 0 and out["status"] == 0


@pytest.mark.parametrize("dev", [0, 1], ids=["host", "device"])
def test_flexible_varn_bput_subarray(gpu, tmp_path, dev):
    """ncmpi_put_varn_all / ncmpi_bput_vara / ncmpi_iput_varn with an MPI
    subarray buftype (the interior of a ghosted 10 x 14 int array), from
    host and hipMalloc'ed buffers: file bytes = MPI_Pack order (the interior,
    row-major) through the oracle's putn; NC_ERANGE from int -> NC_SHORT is
    returned by bput at post and not again by wait (ncmpio_i_getput.m4:
    266-310); get_varn / iget_varn into subarray buffers keep the ghosts
    (checked in api_check)"""
    nc = str(tmp_path / "fd.nc")
    out = _json(capi.run([capi.exe("api_check"), "flexdev", nc, str(dev)]))
    assert out["errors"] == 0
    assert out["bput"] == T.NC_ERANGE and out["wait_status"] == [0, 0]
    vals = ((np.arange(96, dtype=np.int64) * 7919) % 80000 - 40000).astype(np.int32)
    raw = open(nc, "rb").read()
    h = cdfparse.parse_cdf(raw)
    ora = OracleConv()
    for name, xt in (("a", T.NC_INT), ("b", T.NC_SHORT), ("c", T.NC_DOUBLE)):
        exp, st = ora.putn(5, xt, vals, T.ITYPE_INT, T.fill_bytes(xt))
        assert st == (T.NC_ERANGE if xt == T.NC_SHORT else 0)
        assert _var_bytes(raw, h, name) == exp, name
