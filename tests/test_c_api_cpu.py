"""The public ncmpi_* boundary without a GPU (CPU).

libpnetcdf.so (include/pnetcdf.h, include/pncx_dispatch.h) restates the
reference's dispatcher and driver table; everything here runs before any
conversion, so it needs no GPU:
  - every prototype of include/pnetcdf.h is exported, and the header is the
    generator's current output;
  - struct PNC_driver has the reference's member order and signatures
    (src/include/dispatch.h:63-125) and the reference's own benchmark
    benchmarks/C/pnetcdf_put_vara.c compiles against include/pnetcdf.h (both
    read /root/reference, so they skip where it is absent);
  - argument/mode errors of a C program on the API equal the reference's
    codes (var_getput.m4 sanity_check / check_start_count_stride, file.c,
    attr_getput.m4, variable.c, dimension.c);
  - a header defined on 1, 2 and 3 ranks is byte-identical (rank 0 writes it);
  - ncmpii_need_convert through libpncx_ncmpii.so with real MPI_Datatypes
    equals the oracle for every format x xtype x MPI type.
"""
import ctypes
import os
import re
import subprocess
import sys

import pytest

from pnetcdf_amd import nctypes as T
from tests import capi, cdfparse

ROOT = capi.ROOT
REF = "/root/reference"
HDR = os.path.join(ROOT, "include", "pnetcdf.h")


def test_generated_header_is_current():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_pnetcdf_h
    assert open(HDR).read() == gen_pnetcdf_h.gen(), "include/pnetcdf.h is stale: run tools/gen_pnetcdf_h.py"


def _declared():
    return sorted(set(re.findall(r"^(?:int|const char \*)\s*(ncmpi_\w+)\(", open(HDR).read(), re.M)))


def test_libpnetcdf_exports_every_prototype():
    names = _declared()
    assert len(names) == 915                      # the reference's pnetcdf.h.in declares 915
    lib = ctypes.CDLL(os.path.join(ROOT, "pnetcdf_amd", "lib", "libpnetcdf.so"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing[:20]
    for n in ("ncmi355x_inq_driver", "pncx_set_driver"):
        assert hasattr(lib, n)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_prototype_set_equals_reference():
    text = open(os.path.join(REF, "src/include/pnetcdf.h.in")).read()
    ref = set(re.findall(r"^(ncmpi_\w+)\(", text, re.M))
    ref |= set(re.findall(r"^PNETCDF_PUBLIC_API [^(\n]*?\b(ncmpi_\w+)\(", text, re.M))
    assert ref == set(_declared())


def _members(text):
    body = text[text.index("struct PNC_driver {"):]
    body = body[:body.index("};")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    decls = [re.sub(r"\s+", "", d) for d in body.split(";") if "(*" in d]
    return decls


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_driver_table_matches_reference():
    ours = _members(open(os.path.join(ROOT, "include", "pncx_dispatch.h")).read())
    ref = _members(open(os.path.join(REF, "src/include/dispatch.h")).read())
    assert len(ours) == len(ref) == 47
    assert ours == ref


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present")
def test_reference_benchmark_compiles_against_our_header(tmp_path):
    src = os.path.join(REF, "benchmarks", "C", "pnetcdf_put_vara.c")
    r = subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Werror", f"-I{ROOT}/include", "-I/opt/conda/include",
                        src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


# the reference's codes for the calls api_check.c's "errors" mode makes
EXPECTED_ERRORS = {
    "create_bad_path": -223, "create_both_formats": -228, "create_netcdf4": -128, "create": 0,
    "noclobber_exists": -35, "def_dim": 0, "def_dim_x": 0, "def_dim_second_unlimited": -54,
    "def_dim_name_in_use": -42, "def_var_cdf1_int64": -232, "def_var_badtype": -45, "def_var": 0,
    "def_var_text": 0, "def_var_rec": 0, "put_in_define_mode": -39, "inq_bad_ncid": -33,
    "put_att_echar": -56, "put_att_strict_cdf2": -232, "put_att_negative_len": -36, "put_att_text": 0,
    "inq_att_missing": -43, "enddef": 0, "enddef_again": -38, "def_dim_in_data_mode": -38,
    "put_global": -50, "put_bad_varid": -49, "put_indep_in_coll_mode": -202, "put_text_into_int": -56,
    "put_int_into_text": -56, "put_start_out_of_bound": -40, "put_start_negative": -40, "put_edge": -57,
    "put_stride_zero": -58, "get_rec_beyond_numrecs": -40, "put_vara_null_count": -57,
    "flex_ignore_derived": -36, "bput_no_buffer": -217, "wait_indep_in_coll_mode": -202,
    "begin_indep": 0, "put_coll_in_indep_mode": -203, "wait_all_in_indep_mode": -203, "end_indep": 0,
    "redef": 0, "redef_again": -39, "del_att": 0, "enddef2": 0, "del_att_data_mode": -38,
    "vard_deprecated": -214, "malloc_size_disabled": -222, "close": 0, "close_again": -33,
    "open_missing": -220, "open_ro": 0, "put_read_only": -37, "redef_read_only": -37, "inq": 0,
    "inq_format": 0, "inq_dim": 0, "inq_varname": 0, "inq_attlen": -43, "inq_num_rec_vars": 0,
    "close_ro": 0,
}


def test_dispatcher_error_codes(tmp_path):
    r = capi.run([capi.exe("api_check"), "errors", str(tmp_path)])
    got, extra = {}, {}
    for line in r.stdout.splitlines():
        k, *v = line.split()
        if k in EXPECTED_ERRORS:
            got[k] = int(v[0])
        else:
            extra[k] = v
    assert got == EXPECTED_ERRORS
    assert extra["inq_values"] == ["2", "3", "0", "0"]       # ndims nvars ngatts unlimdimid
    assert extra["format"] == ["1"] and extra["dim1"] == ["x", "4"] and extra["var2"] == ["r"]
    assert extra["num_rec_vars"] == ["1"]


@pytest.mark.skipif(not capi.have_mpiexec(), reason="mpiexec not available")
def test_header_identical_on_1_2_3_ranks(tmp_path):
    paths = []
    for n in (1, 2, 3):
        p = str(tmp_path / f"h{n}.nc")
        capi.run([capi.exe("api_check"), "header", p], nprocs=n)
        paths.append(p)
    raw = [open(p, "rb").read() for p in paths]
    assert raw[0] == raw[1] == raw[2]
    h = cdfparse.parse_cdf(raw[0])
    assert h["version"] == 2 and [d[0] for d in h["dims"]] == ["time", "lat", "lon"]
    assert [v["name"] for v in h["vars"]] == ["temp", "lat", "flag", "name"]
    assert set(h["gatts"]) == {"title", "history"}


def test_ncmpii_need_convert_with_mpi_datatypes(tmp_path):
    """ncmpii_need_convert(format, xtype, MPI_Datatype) through
    libpncx_ncmpii.so for every format x xtype x MPI type, against the
    oracle's restatement of convert_swap.m4:85-116 (an MPI type with no
    conversion itype needs conversion unless the variable is text)."""
    from oracle import oracle as O
    cases, exp = [], []
    for fmt in (1, 2, 5):
        for xt in list(T.NUMERIC_XTYPES) + [T.NC_CHAR]:
            for mi in range(14):
                if xt == T.NC_CHAR and mi != 11:
                    continue                       # the reference asserts itype == MPI_CHAR
                cases.append(capi.case(3, fmt, xt, mi))
                it = capi.MPI_IDX_ITYPE.get(mi, 0)
                exp.append(O.need_convert(fmt, xt, it) if it else (0 if xt == T.NC_CHAR else 1))
    cp, op = str(tmp_path / "c.bin"), str(tmp_path / "o.bin")
    open(cp, "wb").write(b"".join(cases))
    capi.run([capi.exe("ncmpii_check"), "run", cp, op])
    got = [st for st, _ in capi.read_results(op)]
    assert got == exp


def test_ncid_table_under_threads(tmp_path):
    """32 threads of one process create, define, close, reopen, inquire
    and close their own files 300 times each through the public API
    (api_check pthreadhdr; define mode only, so no GPU).  The dispatcher's
    ncid table is guarded by a mutex as the reference's is under
    PNETCDF_THREAD_SAFE (src/dispatchers/file.c:30-33,621-703); without it
    this program crashes or reports NC_EBADID within a few iterations.  No
    error, and no file left open.  The data-path restatement of
    tst_pthread.c runs on the GPU (tests/test_gpu_pthread.py)."""
    import json
    r = capi.run([capi.exe("api_check"), "pthreadhdr", str(tmp_path / "thr.nc"), "32", "300"], timeout=120)
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line["errors"] == 0 and line["files_open"] == 0 and line["threads"] == 32
