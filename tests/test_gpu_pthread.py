"""Several threads of one process, each on its own file, through the public
ncmpi_* API (GPU): the reference's test/testcases/tst_pthread.c restated
in tests/mpi/api_check.c (`pthread` mode).  The reference makes its ncid
table thread-safe with a mutex (src/dispatchers/file.c:30-33,621-703); this
library also shares process-wide state between files: the pinned staging
area (g_stage_lock), the device arena, the create/open warm-up thread and
the enddef preload thread (pnetcdf_amd/csrc/pncx_nc.c).

Each of 6 threads creates its file, writes records 0 and 2 of ivar(time, X)
NC_INT and all of dvar(Y, X) NC_DOUBLE, syncs and closes; after a barrier it
opens the next thread's file and reads everything back (the program checks
the values).  Here every file's bytes are compared with the CPU oracle's
putn of the same values at the offsets the program reports.  Sizes: the
reference's NX=4, NY=5, and 1 MiB records (2^18 elements) so that the
threads' staged pipelines overlap; host and hipMalloc'ed buffers;
collective and independent mode."""
import json
import os

import numpy as np
import pytest

from pnetcdf_amd import nctypes as T
from tests import capi
from tests.converters import OracleConv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"


def _ival(tid, r, nx):
    i = np.arange(nx, dtype=np.uint64)
    return ((np.uint64(tid) * np.uint64(1000003) + np.uint64(r) * np.uint64(7919) + i)
            & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)


def _dval(tid, n):
    return tid + 0.5 * np.arange(n, dtype=np.float64)


@pytest.mark.parametrize("nx,ny,coll,dev", [(4, 5, 1, 0), (4, 5, 0, 0), (1 << 18, 4, 1, 0),
                                            (1 << 18, 4, 0, 1), (1 << 16, 3, 1, 1)])
def test_six_threads_six_files(gpu, tmp_path, nx, ny, coll, dev):
    nthreads = 6
    prefix = str(tmp_path / "tst_pthread.nc")
    r = capi.run([capi.exe("api_check"), "pthread", prefix, str(nthreads), str(nx), str(ny), str(coll), str(dev)],
                 timeout=240)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    per = {x["thread"]: x for x in lines if "thread" in x}
    (total,) = [x for x in lines if "threads" in x]
    assert total["errors"] == 0 and sorted(per) == list(range(nthreads)), r.stderr[-3000:]
    ora = OracleConv()
    for tid, o in per.items():
        raw = open(o["file"], "rb").read()
        rs = o["recsize"]
        assert rs == nx * 4
        for rec in (0, 2):
            want, st = ora.putn(1, T.NC_INT, _ival(tid, rec, nx), T.ITYPE_INT, T.fill_bytes(T.NC_INT))
            assert st == 0
            off = o["ivar_off"] + rec * rs
            assert raw[off:off + nx * 4] == want, (tid, rec)
        want, st = ora.putn(1, T.NC_DOUBLE, _dval(tid, nx * ny), T.ITYPE_DOUBLE, T.fill_bytes(T.NC_DOUBLE))
        assert st == 0
        assert raw[o["dvar_off"]:o["dvar_off"] + nx * ny * 8] == want, tid
        # numrecs (CDF-1: 4 big-endian bytes at offset 4) counts the third record
        assert int.from_bytes(raw[4:8], "big") == 3
