"""The create/open warm-up (round 5): ncmpi_create and
ncmpi_open start the HIP runtime on the calling thread and set up the device
context, the pinned staging area, the I/O pool and the kernel files' code
objects on a thread that enddef, the first data call and close wait for.  It
must not change a byte, must leave the first put of the process cheaper than
without it (the reference's benchmark times the put loop,
benchmarks/C/pnetcdf_put_vara.c:191-217), and a process that exits while it
still runs must exit cleanly."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from tests import capi

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHM = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"


def _c1first(path, warm, dev, n=(1 << 18) + 5, nrec=4):
    env = dict(os.environ, PNCX_WARM=str(warm))
    r = capi.run([capi.exe("api_check"), "c1first", path, str(n), str(nrec), str(dev)], env=env)
    out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(out) == 1, r.stdout
    return out[0], open(path, "rb").read()


@pytest.mark.parametrize("dev", [0, 1], ids=["host", "device"])
def test_warmup_same_file_and_cheaper_first_put(dev):
    """the same file bytes and read-back checks with the warm-up off and on;
    with it on, the process's first put is cheaper than with it off (the
    setup moved into create..enddef)"""
    p = os.path.join(SHM, f"pncx_warm_{os.getpid()}_{dev}.nc")
    try:
        off, raw_off = _c1first(p, 0, dev)
        on, raw_on = _c1first(p, 1, dev)
    finally:
        if os.path.exists(p):
            os.unlink(p)
    assert off["errors"] == 0 and on["errors"] == 0
    assert raw_off == raw_on
    print(f"first put: warm-up off {off['put_first_ms']:.2f} ms (create..enddef {off['create_to_enddef_ms']:.2f}), "
          f"on {on['put_first_ms']:.2f} ms (create..enddef {on['create_to_enddef_ms']:.2f})")
    assert on["put_first_ms"] < off["put_first_ms"]


EXIT_EARLY = r"""
import sys
sys.path.insert(0, {root!r})
from pnetcdf_amd import ncfile as N
err, ncid = N.{call}
assert err == 0, err
# no enddef, no close: the process ends while the warm-up may still run
"""


@pytest.mark.parametrize("call", ["create", "open"])
def test_exit_while_warming_up(call):
    """create (or open) and exit at once, without enddef or close: the
    process exits with status 0 (the warm-up thread is joined by an exit
    handler that runs before the HIP runtime's own)"""
    path = os.path.join(SHM, f"pncx_warm_exit_{os.getpid()}.nc")
    from pnetcdf_amd import ncfile as N
    err, ncid = N.create(path, N.NC_64BIT_DATA)
    assert err == 0
    N.def_dim(ncid, "x", 4)
    assert N.enddef(ncid) == 0 and N.close(ncid) == 0
    try:
        expr = f"create({path!r}, N.NC_64BIT_DATA)" if call == "create" else f"open({path!r}, 0)"
        r = subprocess.run([sys.executable, "-c", EXIT_EARLY.format(root=ROOT, call=expr)], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
    finally:
        os.unlink(path)


def test_warmup_entry_point():
    """pncx_warmup on its own: NC_NOERR on a GPU, and twice is harmless"""
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    assert lib.pncx_warmup() == 0
    assert lib.pncx_warmup() == 0
