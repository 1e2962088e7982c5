"""File windows against the CPU's view of the file (round 6: the file-layer
fuzz saw, through pread, data a window put had stored 16 or 32 pages away
from where it belonged, while reads through the same window agreed).

One tmpfs file with a 4 Mi-element NC_INT variable; each round puts a
random range twice with fresh data (the second touch of a range goes
through a file window, DESIGN.md "file windows"), then reads the range back
with os.pread and compares it with the data; sometimes it also reads the
range through the library (window) and puts elsewhere to move the window.
Mismatches are reported with the element shift that explains them.
    python tools/window_probe.py [rounds]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if not os.environ.get("PNCX_NO_TORCH"):
    import torch  # noqa: E402,F401

from pnetcdf_amd import nctypes as T  # noqa: E402
from pnetcdf_amd import ncfile as N  # noqa: E402
from tests import cdfparse  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 200
n = 4 << 20
path = f"/dev/shm/pncx_window_probe_{os.getpid()}.nc"
err, ncid = N.create(path, N.NC_64BIT_DATA)
assert err == 0
N.def_dim(ncid, "x", n)
N.def_var(ncid, "v", T.NC_INT, [0])
assert N.set_fill(ncid, N.NC_FILL)[0] == 0          # the whole variable exists from enddef on
assert N.enddef(ncid) == 0
assert N.sync(ncid) == 0
begin = None
fd = os.open(path, os.O_RDONLY)
rng = np.random.default_rng(3)
model = np.full(n, -2147483647, np.int32)            # NC_INT's default fill
report = {"rounds": rounds, "bad": 0, "examples": [], "window_gets_bad": 0}


def var_begin():
    raw = open(path, "rb").read(1 << 16)
    return cdfparse.parse_cdf(raw + b"\0" * 64)["vars"][0]["begin"]


def check(r, what):
    global begin
    if begin is None:
        begin = var_begin()
    raw = np.frombuffer(os.pread(fd, n * 4, begin), ">i4").astype(np.int32)
    if not np.array_equal(raw, model):
        bad = np.nonzero(raw != model)[0]
        i = int(bad[0])
        hits = np.nonzero(model == raw[i])[0]
        report["bad"] += 1
        report["examples"].append({"round": r, "after": what, "nbad": int(bad.size), "first": i,
                                   "shift": [int(i - h) for h in hits[:3]]})
        model[:] = raw                       # continue from the file's content
        return False
    return True


for r in range(rounds):
    c = int(rng.integers(1 << 18, 1 << 21))
    s = int(rng.integers(0, n - c))
    for touch in range(2):
        vals = rng.integers(-(1 << 31), (1 << 31) - 1, c, dtype=np.int64).astype(np.int32)
        assert N.put_var(ncid, 0, vals, [s], [c]) == 0
        model[s:s + c] = vals
        check(r, f"put {touch} [{s}, {s + c})")
    if rng.random() < 0.5:
        out = np.zeros(c, np.int32)
        assert N.get_var(ncid, 0, out, [s], [c]) == 0
        if not np.array_equal(out, model[s:s + c]):
            report["window_gets_bad"] += 1
    if len(report["examples"]) >= 10:
        break
N.close(ncid)
os.close(fd)
os.unlink(path)
print(json.dumps(report), flush=True)
