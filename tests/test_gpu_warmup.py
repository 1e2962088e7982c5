"""The create/open warm-up and the enddef preload.

ncmpi_create, and ncmpi_open of a writable file, start a thread that
starts the HIP runtime itself and sets up the pinned staging area and the
I/O pool; enddef and the first data call wait for it and then, on the
caller's own device, set up the device context and load the same-type swap
kernels' code object (pncx_warmup).  close only joins the thread.  A
read-only open starts nothing: a program that only reads the header never
touches the device.  enddef then loads the put and get code objects of the
external types the file defines (pncx_preload_xtypes), so a cross-type
first put (put_vara_double into NC_INT) does not pay its type's load.

None of it may change a byte; the first put of the process must be cheaper
with the warm-up than without (the reference's benchmark times the put
loop, benchmarks/C/pnetcdf_put_vara.c:191-217), and a process that exits
while the thread still runs must exit cleanly."""
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


def _c1first(path, warm, dev, n=(1 << 18) + 5, nrec=4, itype=None, preload=None):
    env = dict(os.environ, PNCX_WARM=str(warm))
    if preload is not None:
        env["PNCX_PRELOAD"] = str(preload)
    r = capi.run([capi.exe("api_check"), "c1first", path, str(n), str(nrec), str(dev)] + ([itype] if itype else []),
                 env=env)
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


@pytest.mark.parametrize("dev", [0, 1], ids=["host", "device"])
def test_cross_type_first_put_after_preload(dev):
    """a first put that converts (double -> NC_INT) right after enddef costs
    at most twice a same-type first put (int -> NC_INT): enddef loaded the
    NC_INT put/get code object.  The same run without the preload is
    printed for comparison.  Files equal the same-type run's values."""
    p = os.path.join(SHM, f"pncx_preload_{os.getpid()}_{dev}.nc")
    res = {}
    try:
        for key, itype, pre in (("int", None, 1), ("double", "double", 1), ("double_nopreload", "double", 0),
                                ("int2", None, 1), ("double2", "double", 1)):
            o, raw = _c1first(p, 1, dev, itype=itype, preload=pre)
            assert o["errors"] == 0, key
            res[key] = (o, raw)
    finally:
        if os.path.exists(p):
            os.unlink(p)
    for k, (o, _) in res.items():
        print(f"{k}: put_first {o['put_first_ms']:.2f} ms, create..enddef {o['create_to_enddef_ms']:.2f} ms, "
              f"put median {o['put_ms_median']:.3f} ms")
    same = min(res["int"][0]["put_first_ms"], res["int2"][0]["put_first_ms"])
    cross = min(res["double"][0]["put_first_ms"], res["double2"][0]["put_first_ms"])
    assert cross <= 2.0 * same, (cross, same)
    # the double values are the int values: the records hold the same bytes
    assert res["double"][1] == res["int"][1]


RO_OPEN = r"""
import os, sys
sys.path.insert(0, {root!r})
from pnetcdf_amd import ncfile as N

def kfd_open():
    for fd in os.listdir("/proc/self/fd"):
        try:
            if os.readlink(f"/proc/self/fd/{{fd}}") == "/dev/kfd":
                return True
        except OSError:
            pass
    return False

err, ncid = N.open({path!r}, {mode})
assert err == 0, err
assert N.inq(ncid)[0] == 0
assert N.close(ncid) == 0
print("KFD", int(kfd_open()))
"""


@pytest.mark.parametrize("mode,expect", [(0, 0), (1, 1)], ids=["read-only", "writable"])
def test_read_only_open_leaves_the_device_alone(mode, expect):
    """open + inq + close: read-only, the process never opens /dev/kfd (the
    HIP runtime is not started); writable (the control), the warm-up has
    started it"""
    path = os.path.join(SHM, f"pncx_ro_{os.getpid()}.nc")
    from pnetcdf_amd import ncfile as N
    err, ncid = N.create(path, N.NC_64BIT_DATA)
    assert err == 0
    N.def_dim(ncid, "x", 4)
    assert N.enddef(ncid) == 0 and N.close(ncid) == 0
    env = dict(os.environ, PNCX_WARM="1")       # the control needs the warm-up on, whatever the suite runs with
    try:
        r = subprocess.run([sys.executable, "-c", RO_OPEN.format(root=ROOT, path=path, mode=mode)],
                           capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        assert f"KFD {expect}" in r.stdout, r.stdout
    finally:
        os.unlink(path)
