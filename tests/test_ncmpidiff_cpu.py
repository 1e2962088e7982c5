"""ncmpidiff restatement (pnetcdf_amd/ncmpidiff.py): header comparison, options
and exit codes without a GPU.  Expected lines are the reference's printf
formats (src/utils/ncmpidiff/ncmpidiff_core.c, cited per case); data
comparison runs on the GPU (tests/test_gpu_ncmpidiff.py)."""
import io
import os
import shutil

import pytest

from pnetcdf_amd import ncfile as N
from pnetcdf_amd import ncmpidiff as D
from pnetcdf_amd import nctypes as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TST = os.path.join(ROOT, "tests", "golden", "tst_file.nc")


def make(path, fmt=N.NC_64BIT_DATA, dims=(("x", 4), ("y", 3)), vars_=(("a", T.NC_INT, (0, 1)),),
         gatt=b"hello", vatt=None):
    err, ncid = N.create(path, fmt)
    assert err == 0
    N.set_fill(ncid, N.NC_NOFILL)
    ids = [N.def_dim(ncid, n, ln)[1] for n, ln in dims]
    for name, xt, dd in vars_:
        N.def_var(ncid, name, xt, [ids[d] for d in dd])
    if gatt is not None:
        N.put_att_text(ncid, N.NC_GLOBAL, "title", gatt)
    if vatt is not None:
        N.put_att_text(ncid, 0, "units", vatt)
    assert N.enddef(ncid) == 0
    assert N.close(ncid) == 0
    return path


def run(*argv):
    out = io.StringIO()
    import sys
    old = sys.stdout
    sys.stdout = out
    try:
        rc = D.main(list(argv))
    finally:
        sys.stdout = old
    return rc, out.getvalue().splitlines()


def test_identical_names_error(capsys):
    """ncmpidiff_core.c:349-353 (and src/utils/ncmpidiff/xfail_runs.sh)"""
    assert D.ncmpidiff_core(TST, TST) == T.NC_EINVAL
    assert "two input file names are identical" in capsys.readouterr().err
    assert D.main([TST, TST]) == 1


def test_missing_file(tmp_path, capsys):
    assert D.main([TST, str(tmp_path / "nope.nc")]) == 1
    assert "ncmpidiff input file" in capsys.readouterr().err


def test_usage_errors():
    assert run(TST)[0] == 1
    assert run("-t", "1e-3", TST, TST + "x")[0] == 1        # -t needs diff,ratio


def test_header_same(tmp_path):
    b = str(tmp_path / "b.nc")
    shutil.copy(TST, b)
    rc, lines = run("-h", TST, b)
    assert rc == 0 and lines == ["Headers of two files are the same"]
    rc, lines = run("-q", "-h", TST, b)
    assert rc == 0 and lines == []


def test_header_differences(tmp_path):
    a = make(str(tmp_path / "a.nc"), gatt=b"hello", vatt=b"m/s")
    b = make(str(tmp_path / "b.nc"), fmt=N.NC_64BIT_OFFSET, dims=(("x", 4), ("y", 5), ("z", 2)),
             vars_=(("a", T.NC_FLOAT, (0, 1)), ("c", T.NC_INT, (2,))), gatt=b"help!", vatt=None)
    rc, lines = run("-h", a, b)
    assert rc == 1
    assert lines == [
        "DIFF: file format (CDF-5) != (CDF-2)",                                   # :362
        "DIFF: number of dimensions (2) != (3)",                                  # :389
        "DIFF: number of variables (1) != (2)",                                   # :398
        "ncmpidiff -h %s %s" % (a, b),                                            # PRINT_CMD_OPTS
        'DIFF: global attribute "title" of type NC_CHAR at element 3 of value "hello" vs "help!"',  # :88-91
        'DIFF: dimension "y" length (3) != (5)',                                  # :520
        'DIFF: dimension "z" defined in %s not found in %s' % (b, a),            # :538
        'DIFF: variable "a" data type (NC_INT) != (NC_FLOAT)',                    # :583
        'DIFF: variable "a" of type "NC_INT" dimension 1\'s length (3) != (5)',   # :625
        'DIFF: variable "a" number of attributes (1) != (0)',                     # :637
        'DIFF: variable "a" attribute "units" defined in %s not found in %s' % (a, b),  # :655
        'DIFF: variable "c" defined in %s not found in %s' % (b, a),             # :728
        "Number of differences in header 11",                                     # :944
    ]
    # -q drops the header DIFF lines but not content differences (PRINT_CMD_OPTS path)
    rc, lines = run("-q", "-h", a, b)
    assert rc == 1 and lines == ["ncmpidiff -q -h %s %s" % (a, b),
                                 'DIFF: global attribute "title" of type NC_CHAR at element 3 of value "hello" vs "help!"']


def test_variable_list_structure_differences(tmp_path):
    """-v without -h: structural differences are reported by the data pass
    (ncmpidiff_core.c:753-849) and the variable that is missing is a WARN"""
    a = make(str(tmp_path / "a.nc"))
    b = make(str(tmp_path / "b.nc"), vars_=(("a", T.NC_SHORT, (0, 1)),))
    rc, lines = run("-v", "a,zz", a, b)
    assert rc == 1
    assert lines == ['DIFF: variable "a" data type (NC_INT) != (NC_SHORT)',
                     'WARN: variable "zz" defined in %s not found in %s' % (b, a),
                     "Compared variables(s) has 2 differences"]


def test_verbose_same_lines(tmp_path):
    b = str(tmp_path / "b.nc")
    shutil.copy(TST, b)
    rc, lines = run("-b", "-h", TST, b)
    assert rc == 0
    assert lines[:5] == ["First  file: %s" % TST, "Second file: %s" % b, "SAME: number of dimensions (3)",
                         "SAME: number of variables (2)", "SAME: number of global attributes (1)"]
    assert lines[-1] == "Headers of two files are the same"
