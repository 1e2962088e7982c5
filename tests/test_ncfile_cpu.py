"""File-level layer on CPU: the CDF header codec and the no-conversion data
paths (text and 1-byte variables), pinned by the reference's own fixture
files (tests/golden/cdf, tests/golden/tst_file.nc, copied data files of the
reference's tests) and by an independent reader (scipy.io.netcdf_file).

Expected errors for the corrupted fixtures follow the reference's test
lists: src/utils/ncvalidator/Makefile.am:29-74 (ENULLPAD / EMAXVARS /
EUNLIMIT / ENOTNC / EVARSIZE groups checked by ncvalidator and tst_open.c),
test/cdf_format/tst_corrupt.c:91-154 (EBADTYPE, EMAXDIMS, EBADDIM,
EMAXATTS), test/cdf_format/tst_open_cdf5.c:10-29 (bad_begin -> ENOTNC),
test/cdf_format/test_inq_format.c:20-70 (formats; NC_ENOTBUILT for HDF5).
ncmpi_open checks no header padding (PNETCDF_NULL_BYTE_HEADER_PADDING is 0 by
default, configure.ac:2517-2527); ncvalidator does (pncx_nc_validate).
"""
import os

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from pnetcdf_amd import ncfile as N
from tests import cdfparse

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CDF = os.path.join(GOLD, "cdf")


def _expect_open(name):
    base = name.split(".")[0]
    table = {
        "bad_begin": N.NC_ENOTNC, "bad_dimid": N.NC_EBADDIM, "bad_xtype": N.NC_EBADTYPE,
        "bad_ndims": N.NC_EMAXDIMS, "bad_nattrs": N.NC_EMAXATTS, "bad_nvars": N.NC_EMAXVARS,
        "bad_unlimited": N.NC_EUNLIMIT, "bad_magic": N.NC_ENOTNC,
        "bad_large_fixed_var": N.NC_EVARSIZE, "bad_large_rec_2_vars": N.NC_EVARSIZE,
        "bad_large_rec_var": N.NC_EVARSIZE, "pad_superblock": N.NC_ENOTBUILT, "test_cdf": N.NC_NOERR,
    }
    if base.startswith("bad_tag_"):
        return N.NC_ENOTNC, N.NC_ENOTNC
    if base.startswith("bad_padding_"):
        return N.NC_NOERR, N.NC_ENULLPAD
    if base == "test_cdf" and name[-1] in "34":
        return N.NC_ENOTBUILT, N.NC_ENOTNC3
    e = table[base]
    return e, (N.NC_ENOTNC3 if e == N.NC_ENOTBUILT else e)


FIXTURES = sorted(os.listdir(CDF))


def test_fixture_set_complete():
    assert len(FIXTURES) == 59


@pytest.mark.parametrize("name", FIXTURES)
def test_reference_fixture_open_and_validate(name):
    path = os.path.join(CDF, name)
    exp_open, exp_valid = _expect_open(name)
    err, ncid = N.open(path)
    assert err == exp_open, (name, N.strerror(err), N.strerror(exp_open))
    if err == N.NC_NOERR:
        assert N.close(ncid) == N.NC_NOERR
    assert N.validate(path) == exp_valid, (name, N.strerror(N.validate(path)))


@pytest.mark.parametrize("ver", [1, 2, 3, 4, 5])
def test_reference_inq_format(ver):
    """test/cdf_format/test_inq_format.c: format of test_cdf.nc<ver>"""
    path = os.path.join(CDF, f"test_cdf.nc{ver}")
    err, fmt = N.inq_file_format(path)
    assert err == 0
    if ver in (3, 4):         # HDF5 files: NETCDF4, not distinguished from classic model
        assert fmt == N.NC_FORMAT_NETCDF4
        assert N.open(path)[0] == N.NC_ENOTBUILT
        return
    assert fmt == ver
    err, ncid = N.open(path)
    assert err == 0
    assert N.inq_format(ncid) == (0, ver)
    assert N.close(ncid) == 0


@pytest.mark.parametrize("ver,cmode", [(1, 0), (2, N.NC_64BIT_OFFSET), (5, N.NC_64BIT_DATA)])
def test_empty_file_byte_parity(tmp_path, ver, cmode):
    """create + close of an empty dataset reproduces the reference-written
    test_cdf.nc<ver> byte for byte (ABSENT lists, numrecs width)"""
    p = str(tmp_path / f"e{ver}.nc")
    err, ncid = N.create(p, cmode)
    assert err == 0
    assert N.close(ncid) == 0
    assert open(p, "rb").read() == open(os.path.join(CDF, f"test_cdf.nc{ver}"), "rb").read()


def _tst_file_schema(p):
    err, ncid = N.create(p, 0)
    assert err == 0
    assert N.def_dim(ncid, "time", N.NC_UNLIMITED) == (0, 0)
    assert N.def_dim(ncid, "Y", 4) == (0, 1)
    assert N.def_dim(ncid, "X", 12) == (0, 2)
    assert N.put_att_text(ncid, N.NC_GLOBAL, "history", "Mon Aug 13 21:27:48 2018") == 0
    assert N.def_var(ncid, "rec_var", T.NC_FLOAT, [0, 2]) == (0, 0)
    assert N.def_var(ncid, "fix_var", T.NC_FLOAT, [1, 2]) == (0, 1)
    assert N.enddef(ncid) == 0
    return ncid


def test_tst_file_header_byte_parity(tmp_path):
    """Same definitions as the reference-written ncmpidiff fixture give the
    same header bytes and the same layout (v_align 512, record section after
    the fixed variable though rec_var is defined first, recsize 48)."""
    ref = open(os.path.join(GOLD, "tst_file.nc"), "rb").read()
    p = str(tmp_path / "t.nc")
    ncid = _tst_file_schema(p)
    assert N.inq_header_size(ncid) == (0, 200)
    assert N.inq_header_extent(ncid) == (0, 512)
    assert N.inq_varoffset(ncid, 0) == (0, 704)
    assert N.inq_varoffset(ncid, 1) == (0, 512)
    assert N.inq_recsize(ncid) == (0, 48)
    assert N.sync_numrecs(ncid, 2) == 0
    assert N.close(ncid) == 0
    got = open(p, "rb").read()
    assert len(got) == 200 and got == ref[:200]          # padding to 512 is not written
    assert ref[200:512] == bytes(312)


def test_open_tst_file_metadata():
    path = os.path.join(GOLD, "tst_file.nc")
    ref = cdfparse.parse_cdf(open(path, "rb").read())
    err, ncid = N.open(path)
    assert err == 0
    err, ndims, nvars, ngatts, unlim = N.inq(ncid)
    assert (ndims, nvars, ngatts, unlim) == (3, 2, 1, 0)
    for i, (name, size) in enumerate(ref["dims"]):
        assert N.inq_dim(ncid, i) == (0, name, ref["numrecs"] if size == 0 else size)
    for i, v in enumerate(ref["vars"]):
        err, name, xt, dims, natts = N.inq_var(ncid, i)
        assert (name, xt, dims, natts) == (v["name"], v["xtype"], v["dimids"], 0)
        assert N.inq_varoffset(ncid, i) == (0, v["begin"])
    assert N.get_att(ncid, N.NC_GLOBAL, "history") == (0, b"Mon Aug 13 21:27:48 2018")
    assert N.inq_attname(ncid, N.NC_GLOBAL, 0) == (0, "history")
    assert N.get_att(ncid, N.NC_GLOBAL, "nope")[0] == N.NC_ENOTATT
    assert N.inq_varid(ncid, "fix_var") == (0, 1)
    assert N.inq_dimid(ncid, "X") == (0, 2)
    assert N.close(ncid) == 0


def test_define_mode_errors(tmp_path):
    """dispatchers/dimension.c:30-110, variable.c:40-140 checks"""
    err, ncid = N.create(str(tmp_path / "d.nc"), 0)
    assert N.def_dim(ncid, "t", N.NC_UNLIMITED) == (0, 0)
    assert N.def_dim(ncid, "t2", N.NC_UNLIMITED)[0] == N.NC_EUNLIMIT
    assert N.def_dim(ncid, "t", 5)[0] == N.NC_ENAMEINUSE
    assert N.def_dim(ncid, "", 5)[0] == N.NC_EBADNAME
    assert N.def_dim(ncid, "a/b", 5)[0] == N.NC_EBADNAME
    assert N.def_dim(ncid, "trailing ", 5)[0] == N.NC_EBADNAME
    assert N.def_dim(ncid, "-x", 5)[0] == N.NC_EBADNAME
    assert N.def_dim(ncid, "x" * 257, 5)[0] == N.NC_EMAXNAME
    assert N.def_dim(ncid, "big", 2**31)[0] == N.NC_EDIMSIZE      # CDF-1 limit
    assert N.def_dim(ncid, "x", 3) == (0, 1)
    assert N.def_var(ncid, "v", T.NC_INT64, [1])[0] == N.NC_ESTRICTCDF2
    assert N.def_var(ncid, "v", 0, [1])[0] == N.NC_EBADTYPE
    assert N.def_var(ncid, "v", T.NC_INT, [7])[0] == N.NC_EBADDIM
    assert N.def_var(ncid, "v", T.NC_INT, [1, 0])[0] == N.NC_EUNLIMPOS
    assert N.def_var(ncid, "v", T.NC_INT, [0, 1]) == (0, 0)
    assert N.def_var(ncid, "v", T.NC_INT, [1])[0] == N.NC_ENAMEINUSE
    assert N.put_att(ncid, 0, "_FillValue", T.NC_SHORT, np.array([1], np.int16)) == N.NC_EBADTYPE
    assert N.put_att_text(ncid, 5, "a", "x") == N.NC_ENOTVAR
    assert N.put_att(ncid, N.NC_GLOBAL, "a", T.NC_CHAR, np.array([1], np.int32)) == N.NC_ECHAR
    assert N.put_var(ncid, 0, np.zeros(3, np.int32), [0, 0], [1, 3]) == N.NC_EINDEFINE
    assert N.enddef(ncid) == 0
    assert N.enddef(ncid) == N.NC_ENOTINDEFINE
    assert N.def_dim(ncid, "y", 3)[0] == N.NC_ENOTINDEFINE
    assert N.close(ncid) == 0
    assert N.close(ncid) == N.NC_EBADID
    # NOCLOBBER on an existing file, bad cmode
    assert N.create(str(tmp_path / "d.nc"), N.NC_NOCLOBBER)[0] == N.NC_EEXIST
    assert N.create(str(tmp_path / "e.nc"), N.NC_64BIT_DATA | N.NC_64BIT_OFFSET)[0] == N.NC_EINVAL_CMODE
    assert N.open(str(tmp_path / "missing.nc"))[0] == N.NC_ENOENT


def _text_file(p, cmode=N.NC_64BIT_OFFSET):
    err, ncid = N.create(p, cmode)
    assert err == 0
    N.def_dim(ncid, "time", N.NC_UNLIMITED)
    N.def_dim(ncid, "n", 10)
    N.def_dim(ncid, "m", 6)
    assert N.def_var(ncid, "txt", T.NC_CHAR, [1, 2]) == (0, 0)         # fixed (10, 6)
    assert N.def_var(ncid, "rtxt", T.NC_CHAR, [0, 2]) == (0, 1)        # record (time, 6)
    assert N.def_var(ncid, "b", T.NC_BYTE, [1]) == (0, 2)              # fixed byte, schar -> no convert
    assert N.def_var(ncid, "rb", T.NC_BYTE, [0]) == (0, 3)             # record byte
    assert N.enddef(ncid) == 0
    return ncid


def _chars(s):
    return np.frombuffer(s.encode(), dtype="S1").copy()


def test_text_and_byte_roundtrip(tmp_path):
    """data path without conversion: byte placement checked against
    independently computed offsets"""
    p = str(tmp_path / "t.nc")
    ncid = _text_file(p)
    full = np.frombuffer(bytes(range(65, 65 + 60)), dtype="S1").copy()
    assert N.put_var(ncid, 0, full) == 0                               # whole var
    assert N.put_var(ncid, 0, _chars("zz"), [3, 2], [1, 2]) == 0       # vara
    assert N.put_var(ncid, 0, _chars("Q"), [9, 5]) == 0                # var1
    assert N.put_var(ncid, 1, _chars("abcdefghijkl"), [1, 0], [2, 6]) == 0   # records 1..2
    bvals = np.arange(-5, 5, dtype=np.int8)
    assert N.put_var(ncid, 2, bvals[::2].copy(), [0], [5], [2]) == 0  # vars, stride 2
    assert N.put_var(ncid, 3, np.array([7, -8, 9], np.int8), [4], [3]) == 0
    err, ndims, nvars, ngatts, unlim = N.inq(ncid)
    assert N.inq_dim(ncid, 0)[2] == 7                                   # numrecs grew to 4+3
    out = np.zeros(60, "S1")
    assert N.get_var(ncid, 0, out) == 0
    exp = full.copy().reshape(10, 6)
    exp[3, 2:4] = [b"z", b"z"]
    exp[9, 5] = b"Q"
    assert out.tobytes() == exp.tobytes()
    o2 = np.zeros(6, "S1")
    assert N.get_var(ncid, 1, o2, [2, 0], [1, 6]) == 0
    assert o2.tobytes() == b"ghijkl"
    ob = np.zeros(5, np.int8)
    assert N.get_var(ncid, 2, ob, [0], [5], [2]) == 0
    assert list(ob) == list(bvals[::2])
    assert N.close(ncid) == 0
    # bytes on disk, offsets from the independent parser
    raw = open(p, "rb").read()
    h = cdfparse.parse_cdf(raw)
    assert h["numrecs"] == 7
    v = {x["name"]: x for x in h["vars"]}
    assert raw[v["txt"]["begin"]:v["txt"]["begin"] + 60] == exp.tobytes()
    rs = h["recsize"]
    r2 = v["rtxt"]["begin"] + 2 * rs
    assert raw[r2:r2 + 6] == b"ghijkl"
    assert raw[v["b"]["begin"]:v["b"]["begin"] + 10:2] == bvals[::2].tobytes()
    assert raw[v["rb"]["begin"] + 5 * rs:v["rb"]["begin"] + 5 * rs + 1] == np.int8(-8).tobytes()
    # reopen read-only: numrecs and data persist; writes refused
    err, ncid = N.open(p)
    assert err == 0 and N.inq_dim(ncid, 0)[2] == 7
    assert N.put_var(ncid, 0, _chars("x"), [0, 0]) == N.NC_EPERM
    o = np.zeros(60, "S1")
    assert N.get_var(ncid, 0, o) == 0 and o.tobytes() == exp.tobytes()
    assert N.close(ncid) == 0


def test_start_count_errors(tmp_path):
    """var_getput.m4:60-237 error order and the relaxed coordinate bound"""
    ncid = _text_file(str(tmp_path / "e.nc"))
    c = _chars("abc")
    assert N.put_var(ncid, 0, c, [10, 0], [0, 3]) == 0                 # start == shape, count 0: ok (relaxed)
    assert N.put_var(ncid, 0, c, [11, 0], [0, 3]) == N.NC_EINVALCOORDS
    assert N.put_var(ncid, 0, c, [-1, 0], [1, 3]) == N.NC_EINVALCOORDS
    assert N.put_var(ncid, 0, c, [10, 0], [1, 3]) == N.NC_EINVALCOORDS
    assert N.put_var(ncid, 0, c, [9, 4], [1, 3]) == N.NC_EEDGE
    assert N.put_var(ncid, 0, c, [0, 0], [1, -3]) == N.NC_ENEGATIVECNT
    assert N.put_var(ncid, 0, c, [0, 0], [1, 3], [1, 0]) == N.NC_ESTRIDE
    assert N.put_var(ncid, 0, c, [0, 0], [1, 3], [1, 3]) == N.NC_EEDGE  # 0 + 2*3 >= 6
    assert N.put_var(ncid, 0, np.zeros(3, np.int32), [0, 0], [1, 3]) == N.NC_ECHAR
    assert N.put_var(ncid, 7, c, [0, 0], [1, 3]) == N.NC_ENOTVAR
    assert N.put_var(ncid, N.NC_GLOBAL, c, [0, 0], [1, 3]) == N.NC_EGLOBAL
    # record variable: puts may extend, gets may not read past numrecs
    assert N.put_var(ncid, 1, c, [5, 0], [1, 3]) == 0
    o = np.zeros(3, "S1")
    assert N.get_var(ncid, 1, o, [6, 0], [1, 3]) == N.NC_EINVALCOORDS
    assert N.get_var(ncid, 1, o, [5, 0], [2, 3]) == N.NC_EEDGE
    assert N.get_var(ncid, 1, o, [5, 0], [1, 3]) == 0 and o.tobytes() == b"abc"
    assert N.close(ncid) == 0


def test_nonblocking_text_cpu(tmp_path):
    """iput/iget posted, then flushed by one wait_all: offset-sorted
    coalesced writes; per-request statuses; cancel; pending at close"""
    p = str(tmp_path / "nb.nc")
    ncid = _text_file(p)
    rows = [_chars(s * 6) for s in "ABCDEFGHIJ"]
    reqs = []
    for r in (7, 2, 9, 0, 5, 1, 8, 3, 6, 4):             # posted out of order
        err, rq = N.iput_var(ncid, 0, rows[r], [r, 0], [1, 6])
        assert err == 0 and rq >= 0
        reqs.append(rq)
    err, rq = N.iput_var(ncid, 1, _chars("r0r0r0r1r1r1"), [0, 0], [2, 6])
    reqs.append(rq)
    assert N.inq_nreqs(ncid) == (0, 11)
    err, st = N.wait_all(ncid, reqs)
    assert err == 0 and st == [0] * 11
    assert N.inq_nreqs(ncid) == (0, 0)
    assert N.inq_dim(ncid, 0)[2] == 2
    outs = [np.zeros(6, "S1") for _ in range(10)]
    greqs = [N.iget_var(ncid, 0, outs[r], [r, 0], [1, 6])[1] for r in range(10)]
    err, st = N.wait_all(ncid, greqs + [12345])
    assert err == N.NC_EINVAL_REQUEST and st[:10] == [0] * 10 and st[10] == N.NC_EINVAL_REQUEST
    assert [o.tobytes() for o in outs] == [(s * 6).encode() for s in "ABCDEFGHIJ"]
    # cancel drops requests; close with pending requests reports NC_EPENDING
    err, rq = N.iput_var(ncid, 0, _chars("######"), [0, 0], [1, 6])
    assert N.cancel(ncid, [rq])[0] == 0 and N.inq_nreqs(ncid) == (0, 0)
    err, rq = N.iput_var(ncid, 0, _chars("######"), [0, 0], [1, 6])
    assert N.close(ncid) == N.NC_EPENDING
    raw = open(p, "rb").read()
    h = cdfparse.parse_cdf(raw)
    b = h["vars"][0]["begin"]
    assert raw[b:b + 60] == "".join(s * 6 for s in "ABCDEFGHIJ").encode()


def test_redef_moves_data(tmp_path):
    """redef + new variables grow the header and the fixed section: existing
    data moves to the new begins (ncmpio_enddef.c move_fixed/record_vars)"""
    p = str(tmp_path / "r.nc")
    ncid = _text_file(p, 0)
    full = np.frombuffer(bytes(range(65, 125)), dtype="S1").copy()
    assert N.put_var(ncid, 0, full) == 0
    assert N.put_var(ncid, 1, _chars("abcdefghijkl"), [0, 0], [2, 6]) == 0
    assert N.put_var(ncid, 3, np.array([1, 2], np.int8), [0], [2]) == 0
    old_off = [N.inq_varoffset(ncid, i)[1] for i in range(4)]
    assert N.redef(ncid) == 0
    for k in range(40):                                   # grow the header past 512 bytes
        assert N.put_att_text(ncid, N.NC_GLOBAL, f"attribute_number_{k:03d}", "x" * 9) == 0
    assert N.def_var(ncid, "later", T.NC_CHAR, [1, 2]) == (0, 4)
    assert N.def_var(ncid, "rlater", T.NC_CHAR, [0, 2]) == (0, 5)
    assert N._enddef(ncid, 0, 0, 0, 0) == 0
    new_off = [N.inq_varoffset(ncid, i)[1] for i in range(6)]
    assert new_off[0] > old_off[0] and new_off[1] > old_off[1]
    o = np.zeros(60, "S1")
    assert N.get_var(ncid, 0, o) == 0 and o.tobytes() == full.tobytes()
    o = np.zeros(12, "S1")
    assert N.get_var(ncid, 1, o, [0, 0], [2, 6]) == 0 and o.tobytes() == b"abcdefghijkl"
    ob = np.zeros(2, np.int8)
    assert N.get_var(ncid, 3, ob, [0], [2]) == 0 and list(ob) == [1, 2]
    assert N.close(ncid) == 0
    h = cdfparse.parse_cdf(open(p, "rb").read())
    assert len(h["gatts"]) == 40 and len(h["vars"]) == 6


def test_attributes_text_and_rename(tmp_path):
    p = str(tmp_path / "a.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", 4)
    N.def_var(ncid, "v", T.NC_CHAR, [0])
    assert N.put_att_text(ncid, 0, "units", "meters") == 0
    assert N.put_att_text(ncid, N.NC_GLOBAL, "title", "") == 0
    assert N.inq_att(ncid, N.NC_GLOBAL, "title") == (0, T.NC_CHAR, 0)
    assert N.rename_att(ncid, 0, "units", "unit") == 0
    assert N.del_att(ncid, N.NC_GLOBAL, "title") == 0
    assert N.del_att(ncid, N.NC_GLOBAL, "title") == N.NC_ENOTATT
    assert N.rename_var(ncid, 0, "w") == 0
    assert N.rename_dim(ncid, 0, "y") == 0
    assert N.enddef(ncid) == 0
    assert N.rename_var(ncid, 0, "longer_name") == N.NC_ENOTINDEFINE
    assert N.rename_var(ncid, 0, "z") == 0                    # shorter: allowed in data mode
    assert N.close(ncid) == 0
    h = cdfparse.parse_cdf(open(p, "rb").read())
    assert h["vars"][0]["name"] == "z" and h["dims"][0][0] == "y"
    err, ncid = N.open(p)
    assert N.get_att(ncid, 0, "unit") == (0, b"meters")
    assert N.close(ncid) == 0


@pytest.mark.parametrize("version", [1, 2])
def test_scipy_cross_read(tmp_path, version):
    """independent third-party check of on-disk layout: scipy writes CDF-1/2
    (with non-null attribute padding, which ncmpi_open accepts), we read its
    header and 1-byte/text data; we write, scipy reads"""
    sio = pytest.importorskip("scipy.io")
    p = str(tmp_path / "s.nc")
    f = sio.netcdf_file(p, "w", version=version)
    f.history = b"made by scipy"
    f.createDimension("t", None)
    f.createDimension("x", 5)
    v = f.createVariable("c", "c", ("t", "x"))
    v[0:2] = np.frombuffer(b"helloworld", dtype="S1").reshape(2, 5)
    b = f.createVariable("b", "b", ("x",))
    b[:] = np.arange(-2, 3, dtype=np.int8)
    f.close()
    err, ncid = N.open(p)
    assert err == 0
    assert N.inq_format(ncid) == (0, version)
    assert N.inq_dim(ncid, 0) == (0, "t", 2)
    o = np.zeros(10, "S1")
    vid = N.inq_varid(ncid, "c")[1]
    assert N.get_var(ncid, vid, o, [0, 0], [2, 5]) == 0 and o.tobytes() == b"helloworld"
    ob = np.zeros(5, np.int8)
    assert N.get_var(ncid, N.inq_varid(ncid, "b")[1], ob) == 0 and list(ob) == [-2, -1, 0, 1, 2]
    assert N.get_att(ncid, N.NC_GLOBAL, "history") == (0, b"made by scipy")
    assert N.close(ncid) == 0
    # ours -> scipy.  Like PnetCDF we never write the padding after the last
    # record's data; scipy reads whole padded records, so the record variable
    # here is 4-byte aligned.
    q = str(tmp_path / "o.nc")
    err, ncid = N.create(q, N.NC_64BIT_OFFSET if version == 2 else 0)
    N.def_dim(ncid, "time", N.NC_UNLIMITED)
    N.def_dim(ncid, "n", 10)
    N.def_dim(ncid, "m", 8)
    N.def_var(ncid, "rtxt", T.NC_CHAR, [0, 2])
    N.def_var(ncid, "b", T.NC_BYTE, [1])
    assert N.enddef(ncid) == 0
    assert N.put_var(ncid, 0, _chars("abcdefghijklmnop"), [0, 0], [2, 8]) == 0
    assert N.put_var(ncid, 1, np.arange(10, dtype=np.int8)) == 0
    assert N.close(ncid) == 0
    g = sio.netcdf_file(q, "r", mmap=False)
    assert g.variables["rtxt"][:].tobytes() == b"abcdefghijklmnop"
    assert list(g.variables["b"][:]) == list(range(10))
    g.close()


def test_numeric_data_fails_loudly_without_gpu(tmp_path):
    """numeric conversion has no CPU path: with no visible GPU the file layer
    returns PNCX_EDEVICE and writes nothing"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: covered by the gpu tests")
    p = str(tmp_path / "g.nc")
    err, ncid = N.create(p, 0)
    N.def_dim(ncid, "x", 4)
    N.def_var(ncid, "v", T.NC_INT, [0])
    assert N.enddef(ncid) == 0
    size0 = os.path.getsize(p)
    assert N.put_var(ncid, 0, np.arange(4, dtype=np.int32)) == N.PNCX_EDEVICE
    assert N.put_att(ncid, N.NC_GLOBAL, "a", T.NC_INT, np.arange(2, dtype=np.int32)) in (N.PNCX_EDEVICE,
                                                                                     N.NC_ENOTINDEFINE)
    assert N.close(ncid) == 0
    assert os.path.getsize(p) == size0


@pytest.mark.parametrize("threads,mmap", [("1", "0"), ("8", "0"), ("8", "1")])
def test_parallel_io_pool_large(tmp_path, threads, mmap):
    """multi-MiB jobs split over the I/O pool (pncx_io.c): byte variables take
    the copy path, so this runs without a GPU; checked against numpy slicing
    of the file bytes (the pool size is fixed per process, so the env value
    only matters for the first data call of the process)"""
    import subprocess
    import sys
    code = f"""
import os, sys, numpy as np
sys.path.insert(0, {repr(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))})
from pnetcdf_amd import ncfile as N, nctypes as T
from tests import cdfparse
p = {repr(str(tmp_path / 'big.nc'))}
err, ncid = N.create(p, N.NC_64BIT_DATA)
N.def_dim(ncid, 't', N.NC_UNLIMITED); N.def_dim(ncid, 'y', 1024); N.def_dim(ncid, 'x', 8192)
N.def_var(ncid, 'b', T.NC_BYTE, [1, 2]); N.def_var(ncid, 'r', T.NC_BYTE, [0, 2])
assert N.enddef(ncid) == 0
a = np.random.default_rng(1).integers(-128, 127, (1024, 8192), dtype=np.int8)
assert N.put_var(ncid, 0, a) == 0
assert N.put_var(ncid, 0, a[100:900:4, 3:8000:5].copy(), [100, 3], [200, 1600], [4, 5]) == 0
recs = np.random.default_rng(2).integers(-128, 127, (64, 8192), dtype=np.int8)
reqs = [N.iput_var(ncid, 1, recs[r], [r, 0], [1, 8192])[1] for r in range(63, -1, -1)]
assert N.wait_all(ncid, reqs)[0] == 0
o = np.zeros((200, 1600), np.int8)
assert N.get_var(ncid, 0, o, [100, 3], [200, 1600], [4, 5]) == 0
assert np.array_equal(o, a[100:900:4, 3:8000:5])
full = np.zeros((1024, 8192), np.int8)
assert N.get_var(ncid, 0, full) == 0 and np.array_equal(full, a)
assert N.close(ncid) == 0
raw = np.fromfile(p, np.uint8)
h = cdfparse.parse_cdf(raw[:4096].tobytes())
b0 = h['vars'][0]['begin']
assert np.array_equal(raw[b0:b0 + a.size].view(np.int8).reshape(1024, 8192), a)
r0, rs = h['vars'][1]['begin'], h['recsize']
for r in (0, 31, 63):
    assert np.array_equal(raw[r0 + r * rs:r0 + r * rs + 8192].view(np.int8), recs[r])
print('ok')
"""
    env = dict(os.environ, PNCX_IO_THREADS=threads, PNCX_IO_MMAP=mmap)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stderr[-2000:]


def test_varn_text_and_byte(tmp_path):
    """ncmpi_put_varn / get_varn / iput_varn (dispatchers/var_getput.m4:426-560):
    several boxes packed in one buffer; var1 boxes (counts[i] None); errors"""
    p = str(tmp_path / "vn.nc")
    ncid = _text_file(p)
    starts = [[0, 0], [4, 1], [9, 5], [1, 3]]          # disjoint boxes (overlap order is undefined)
    counts = [[1, 6], [2, 3], None, [3, 2]]
    buf = _chars("ABCDEF" + "ghijkl" + "Z" + "mnopqr")
    assert N.put_varn(ncid, 0, starts, counts, buf) == 0
    exp = np.full((10, 6), b"\x00", "S1")
    exp[0, 0:6] = list(b"ABCDEF"[i:i + 1] for i in range(6))
    exp[4:6, 1:4] = np.frombuffer(b"ghijkl", "S1").reshape(2, 3)
    exp[9, 5] = b"Z"
    exp[1:4, 3:5] = np.frombuffer(b"mnopqr", "S1").reshape(3, 2)
    out = np.zeros(60, "S1")
    assert N.get_var(ncid, 0, out) == 0 and out.tobytes() == exp.tobytes()
    back = np.zeros(19, "S1")
    assert N.get_varn(ncid, 0, starts, counts, back) == 0 and back.tobytes() == buf.tobytes()
    # nonblocking varn on a record variable: one request id, numrecs grows
    err, rq = N.iput_varn(ncid, 3, [[6], [1], [3]], [[2], [1], [1]], np.array([1, 2, 3, 4], np.int8))
    assert err == 0 and rq >= 0
    err, rq2 = N.iput_var(ncid, 3, np.array([9], np.int8), [0], [1])
    assert N.wait_all(ncid, [rq, rq2]) == (0, [0, 0])
    assert N.inq_dim(ncid, 0)[2] == 8
    o = np.zeros(8, np.int8)
    assert N.get_var(ncid, 3, o, [0], [8]) == 0 and o.tolist() == [9, 3, 0, 4, 0, 0, 1, 2]
    # errors: NULL starts, bad box (nothing posted), zero boxes
    assert N.put_varn(ncid, 0, None, None, buf) == 0                      # num 0: nothing to do
    assert N.lib().pncx_nc_put_varn(ncid, 0, 2, None, None, buf.ctypes.data, T.ITYPE_CHAR) == N.NC_ENULLSTART
    assert N.put_varn(ncid, 0, [[0, 0], [11, 0]], [[1, 2], [1, 2]], buf[:4].copy()) == N.NC_EINVALCOORDS
    assert N.inq_nreqs(ncid) == (0, 0)
    assert N.close(ncid) == 0


def test_bput_attached_buffer(tmp_path):
    """ncmpio_bput.c / ncmpio_i_getput.m4:266-310: bput converts into the
    attached buffer at post time (the caller's buffer may change right
    after), usage accounting, NC_EINSUFFBUF / NC_ENULLABUF /
    NC_EPREVATTACHBUF / NC_EPENDINGBPUT, tail-first release at wait"""
    p = str(tmp_path / "bp.nc")
    ncid = _text_file(p)
    row = _chars("abcdef")
    assert N.bput_var(ncid, 0, row, [0, 0], [1, 6])[0] == N.NC_ENULLABUF
    assert N.buffer_attach(ncid, 20) == 0
    assert N.buffer_attach(ncid, 20) == N.NC_EPREVATTACHBUF
    assert N.inq_buffer_size(ncid) == (0, 20)
    err, r1 = N.bput_var(ncid, 0, row, [0, 0], [1, 6])
    assert err == 0
    row[:] = _chars("XXXXXX")                          # caller reuses its buffer immediately
    err, r2 = N.bput_var(ncid, 0, _chars("ghijkl"), [1, 0], [1, 6])
    assert N.inq_buffer_usage(ncid) == (0, 12)
    assert N.bput_var(ncid, 0, _chars("mnopqrstu"), [2, 0], [1, 9])[0] == N.NC_EEDGE
    assert N.bput_var(ncid, 0, np.zeros(12, "S1"), [2, 0], [2, 6])[0] == N.NC_EINSUFFBUF
    assert N.buffer_detach(ncid) == N.NC_EPENDINGBPUT
    assert N.wait_all(ncid, [r2]) == (0, [0])          # r2 is at the tail: its space comes back
    assert N.inq_buffer_usage(ncid) == (0, 6)
    assert N.wait_all(ncid, [r1]) == (0, [0])
    assert N.inq_buffer_usage(ncid) == (0, 0)
    assert N.buffer_detach(ncid) == 0
    assert N.buffer_detach(ncid) == N.NC_ENULLABUF
    o = np.zeros(12, "S1")
    assert N.get_var(ncid, 0, o, [0, 0], [2, 6]) == 0 and o.tobytes() == b"abcdefghijkl"
    assert N.close(ncid) == 0


def test_header_larger_than_read_chunk(tmp_path):
    """a header past the 256 KiB first read (nc_header_read_chunk_size):
    open reads more instead of decoding zeros"""
    p = str(tmp_path / "bighdr.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", 16)
    N.def_var(ncid, "b", T.NC_BYTE, [0])
    for k in range(2500):
        assert N.put_att_text(ncid, N.NC_GLOBAL, f"attribute_{k:05d}", f"{k:05d}" * 20) == 0
    assert N.enddef(ncid) == 0
    assert N.inq_header_size(ncid)[1] > 300000
    assert N.put_var(ncid, 0, np.arange(16, dtype=np.int8)) == 0
    assert N.close(ncid) == 0
    err, ncid = N.open(p)
    assert err == 0
    assert N.inq(ncid)[3] == 2500
    assert N.get_att(ncid, N.NC_GLOBAL, "attribute_02499") == (0, b"02499" * 20)
    o = np.zeros(16, np.int8)
    assert N.get_var(ncid, 0, o) == 0 and o.tolist() == list(range(16))
    assert N.close(ncid) == 0
    assert N.validate(p) == 0
