"""The C-ABI libraries load and export every declared symbol (CPU, no GPU).

No compute call is made here; host-side metadata functions are checked
against the oracle, and the compute entry points must fail loudly
(PNCX_EDEVICE) when no GPU is visible instead of silently converting on the
CPU.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pnetcdf_amd", "lib", "libpncx.so")
LIB_MPI = os.path.join(ROOT, "pnetcdf_amd", "lib", "libpncx_ncmpii.so")
LIB_MPIDT = os.path.join(ROOT, "pnetcdf_amd", "lib", "libpncx_mpi.so")


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_]+\s*\*?\s*(\w+)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n.startswith(("pncx_", "ncmpii_"))))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True,
                         check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


@pytest.fixture(scope="module")
def built():
    if not all(os.path.exists(p) for p in (LIB, LIB_MPI, LIB_MPIDT)):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "pnetcdf_amd", "csrc")], check=True)
    return True


def test_pncx_h_symbols_exported(built):
    decl = declared("pncx.h")
    assert len(decl) == 51      # + pncx_phases, pncx_phase_name/read, pncx_knob_set/get, pncx_dev_pack/unpack/alloc/free (round 4), pncx_warmup (round 5), pncx_preload_xtypes/pending (round 6)
    missing = [s for s in decl if s not in exported(LIB)]
    assert not missing, missing


def test_conversion_kernels_one_object_per_external_type(built):
    """pncx_kern_put.hip / pncx_kern_get.hip are compiled once per external
    type (Makefile XTS, round 5): every one of the ten types has its put, get,
    batch, fused-batch, imap and opinfo launchers in libpncx.so, and the
    library holds 2 x 10 + 2 gfx950 code objects (swap, diff), so a process
    loads only the types it converts"""
    syms = exported(LIB)
    xts = [T.NC_BYTE, T.NC_SHORT, T.NC_INT, T.NC_FLOAT, T.NC_DOUBLE, T.NC_UBYTE, T.NC_USHORT, T.NC_UINT,
           T.NC_INT64, T.NC_UINT64]
    fams = ["pncxk_put", "pncxk_batch_put", "pncxk_batch_fused_put", "pncxk_imap_put", "pncxk_opinfo_put",
            "pncxk_get", "pncxk_batch_get", "pncxk_batch_fused_get", "pncxk_imap_get", "pncxk_opinfo_get_get"]
    missing = [f"{f}_x{x}" for f in fams for x in xts if f"{f}_x{x}" not in syms]
    assert not missing, missing
    assert not [s for s in syms if s.startswith("pncxk_put_x") and s not in {f"pncxk_put_x{x}" for x in xts}]
    from tests.test_isa_store_hazard import code_objects
    assert len(code_objects(LIB)) == 22


def test_pncx_nc_h_symbols_exported(built):
    """file-level API (include/pncx_nc.h)"""
    decl = declared("pncx_nc.h")
    assert len(decl) == 63          # + create_shared, set_writer, set_numrecs, bput_varn (round 2)
    missing = [s for s in decl if s not in exported(LIB)]
    assert not missing, missing


def test_ncmpii_symbols_exported(built):
    decl = declared("pncx_ncmpii.h")
    # the 22 conversion symbols of common.h:147-221 (+ CHAR put/get, mapper)
    assert {"ncmpii_in_swapn", "ncmpii_need_convert", "ncmpii_putn_NC_DOUBLE",
            "ncmpii_getn_NC_INT", "ncmpii_putn_NC_BYTE", "ncmpii_getn_NC_UINT64"} <= set(decl)
    assert len([d for d in decl if d.startswith("ncmpii_")]) == 24
    missing = [s for s in decl if s not in exported(LIB_MPI)]
    assert not missing, missing


def test_mpi_buftype_symbols_exported(built):
    """flexible API over MPI derived datatypes (include/pncx_mpi.h)"""
    decl = declared("pncx_mpi.h")
    assert set(decl) == {"pncx_mpi_type_flatten", "pncx_mpi_type_commit", "pncx_ncmpi_put_varm",
                         "pncx_ncmpi_get_varm", "pncx_ncmpi_iput_varm", "pncx_ncmpi_iget_varm"}
    missing = [s for s in decl if s not in exported(LIB_MPIDT)]
    assert not missing, missing


def test_library_loads_and_metadata(built):
    from oracle import oracle as O
    L = ctypes.CDLL(LIB)
    L.pncx_version.restype = ctypes.c_char_p
    assert b"gfx950" in L.pncx_version()
    for fmt in (1, 2, 5):
        for xt in T.NUMERIC_XTYPES + [T.NC_CHAR]:
            for it in T.NUMERIC_ITYPES + [T.ITYPE_CHAR]:
                assert L.pncx_need_convert(fmt, xt, it) == O.need_convert(fmt, xt, it)
    for xt in T.NUMERIC_XTYPES:
        assert L.pncx_xlen(xt) == T.xlen(xt)
        for it in T.NUMERIC_ITYPES:
            assert L.pncx_need_swap(xt, it) == O.need_swap(xt, it)
    for it in T.NUMERIC_ITYPES:
        assert L.pncx_ilen(it) == T.ilen(it)
    assert L.pncx_xlen(99) == -1 and L.pncx_ilen(99) == -1


def test_no_cpu_fallback_without_gpu(built):
    """With no visible GPU the host entry points return PNCX_EDEVICE."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: covered by the gpu tests")
    L = ctypes.CDLL(LIB)
    assert L.pncx_device_count() == 0
    buf = np.arange(16, dtype=np.int64)
    keep = buf.copy()
    rc = L.pncx_in_swapn(ctypes.c_void_p(buf.ctypes.data), ctypes.c_longlong(16), 8)
    assert rc == T.PNCX_EDEVICE
    assert np.array_equal(buf, keep)            # untouched: no silent CPU path
    xb = np.zeros(128, np.uint8)
    rc = L.pncx_putn(5, T.NC_INT, ctypes.c_void_p(xb.ctypes.data), ctypes.c_void_p(buf.ctypes.data),
                     ctypes.c_longlong(16), T.ITYPE_LONGLONG, None)
    assert rc == T.PNCX_EDEVICE
    # argument errors are still reported before the device check
    rc = L.pncx_putn(5, 42, ctypes.c_void_p(xb.ctypes.data), ctypes.c_void_p(buf.ctypes.data),
                     ctypes.c_longlong(16), T.ITYPE_INT, None)
    assert rc == T.NC_EBADTYPE
    # the enddef preload (round 6): nothing to load without a device; the
    # pending mask is the request minus NC_CHAR
    mask = (1 << T.NC_INT) | (1 << T.NC_DOUBLE) | (1 << T.NC_CHAR)
    assert L.pncx_preload_xtypes(0, mask) == T.PNCX_EDEVICE
    L.pncx_preload_pending.restype = ctypes.c_uint
    assert L.pncx_preload_pending(0, mask) == (1 << T.NC_INT) | (1 << T.NC_DOUBLE)
    assert L.pncx_preload_pending(-1, mask) == 0
    # batches: a missing segment array is an argument error, also without a device
    st = (ctypes.c_int * 3)()
    assert L.pncx_dev_batch(None, 3, st, None) == T.NC_EINVAL
    assert L.pncx_batch(None, 3, st) == T.NC_EINVAL
    assert L.pncx_dev_batch(None, 0, st, None) == T.NC_NOERR


def test_ncmpii_in_swapn_aborts_without_gpu(built):
    """ncmpii_in_swapn returns void upstream (common.h:151), so a device
    failure cannot be reported: the shim aborts the process rather than
    return with the buffer unswapped (pncx_ncmpii.c).  The child process
    gets SIGABRT and says why."""
    import subprocess
    import sys
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: the call would succeed")
    lib = os.path.join(os.path.dirname(LIB), "libpncx_ncmpii.so")
    code = ("import ctypes, numpy as np\n"
            "L = ctypes.CDLL(%r)\n"
            "b = np.arange(4, dtype=np.int64)\n"
            "L.ncmpii_in_swapn(ctypes.c_void_p(b.ctypes.data), ctypes.c_longlong(4), 8)\n"
            "print('returned')\n" % lib)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == -6, (r.returncode, r.stdout, r.stderr)
    assert "returned" not in r.stdout
    assert "ncmpii_in_swapn" in r.stderr


def test_product_does_not_reference_oracle():
    """The product sources never include, link or load the oracle."""
    for d, _, files in os.walk(os.path.join(ROOT, "pnetcdf_amd")):
        for f in files:
            if f.endswith((".c", ".h", ".hpp", ".hip", ".py", "Makefile")):
                txt = open(os.path.join(d, f)).read()
                for pat in ("import oracle", "from oracle", "liboracle", "orc_", "pncx_oracle"):
                    assert pat not in txt, (os.path.join(d, f), pat)
    for lib in (LIB, LIB_MPI):
        if os.path.exists(lib):
            out = subprocess.run(["readelf", "-d", lib], capture_output=True, text=True).stdout
            assert "oracle" not in out
