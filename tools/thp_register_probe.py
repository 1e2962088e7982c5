"""Do kernels see a host buffer the library registers per call (zero copy)
where the CPU sees it?  (Round 6: the file-layer fuzz found data shifted by
16 or 32 pages after a put through a user buffer the call registered.)

Fresh numpy buffers of a few MiB each round -- numpy asks for transparent
huge pages on large arrays (madvise) -- converted host to host by
pncx_putn / pncx_getn (the library registers both buffers for the call and
the kernel reads and writes them over PCIe), checked against numpy's own
byte swap; any mismatch is reported with the page shift that explains it.
    python tools/thp_register_probe.py [rounds] [mib] [nohuge]
nohuge: madvise(MADV_NOHUGEPAGE) on every buffer before its first touch."""
import ctypes
import json
import mmap
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime with torch, as the tests)

from pnetcdf_amd import nctypes as T  # noqa: E402
from pnetcdf_amd import pncx  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 200
mib = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
nohuge = len(sys.argv) > 3 and sys.argv[3] == "nohuge"
libc = ctypes.CDLL(None)
MADV_NOHUGEPAGE = 15


def fresh(nbytes):
    """a new buffer; nohuge: an anonymous mapping madvised before first touch"""
    if not nohuge:
        return np.empty(nbytes, np.uint8)
    m = mmap.mmap(-1, nbytes + 4096)
    a = np.frombuffer(m, np.uint8)
    libc.madvise(ctypes.c_void_p(a.ctypes.data & ~4095), ctypes.c_size_t(nbytes + 4096), MADV_NOHUGEPAGE)
    return a[:nbytes]


def shift_of(got, want):
    """element shift s with got[i] == want[i - s] at the first bad index, if any"""
    bad = np.nonzero(got != want)[0]
    i = int(bad[0])
    hits = np.nonzero(want == got[i])[0]
    return len(bad), i, [int(i - h) for h in hits[:3]]


rng = np.random.default_rng(1)
n = int(mib * (1 << 20)) // 4
report = {"rounds": rounds, "mib": mib, "nohuge": nohuge, "put_bad": 0, "get_bad": 0, "examples": []}
for r in range(rounds):
    src = fresh(n * 4).view(np.int32)
    src[:] = rng.integers(-(1 << 31), (1 << 31) - 1, n, dtype=np.int64).astype(np.int32)
    want = src.astype(">i4").view(np.int32)
    x = fresh(n * 4)
    x[:] = 0
    assert pncx.putn(5, T.NC_INT, x, src, n, T.ITYPE_INT) == 0
    got = x.view(np.int32)
    if not np.array_equal(got, want):
        report["put_bad"] += 1
        report["examples"].append({"round": r, "dir": "put", "src": hex(src.ctypes.data), "dst": hex(x.ctypes.data),
                                   "bad_shift": shift_of(got, want)})
    back = fresh(n * 8).view(np.float64)
    back[:] = 0
    assert pncx.getn(5, T.NC_INT, x, back, n, T.ITYPE_DOUBLE) == 0
    wb = src.astype(np.float64)
    if not np.array_equal(back, wb):
        report["get_bad"] += 1
        report["examples"].append({"round": r, "dir": "get", "src": hex(x.ctypes.data), "dst": hex(back.ctypes.data),
                                   "bad_shift": shift_of(back, wb)})
    if len(report["examples"]) >= 10:
        break
    del src, x, back
try:
    report["numpy_madvise_hugepage"] = bool(np.core.multiarray._get_madvise_hugepage())
except Exception:
    report["numpy_madvise_hugepage"] = None
try:
    report["anon_huge_kb"] = [int(l.split()[1]) for l in open("/proc/self/smaps_rollup") if l.startswith("AnonHugePages")][0]
    report["thp_enabled"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
except OSError:
    pass
print(json.dumps(report), flush=True)
