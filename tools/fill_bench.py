"""HBM write rate of the fill kernel (pncx_dev_fill, fill_var_buf of
ncmpio_fill.c:89-140) against torch's own fill_ of the same bytes on the same
device.  Algorithmic bytes = nelems * xsize (write only).  HIP events on the
current stream, median of 10."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from pnetcdf_amd import nctypes as T  # noqa: E402
from pnetcdf_amd import pncx  # noqa: E402

GIB = 1 << 30


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[reps // 2]


def main():
    gib = 16
    buf = torch.empty(gib * GIB, dtype=torch.uint8, device="cuda")
    rows = []
    for name, xt in (("NC_DOUBLE", T.NC_DOUBLE), ("NC_FLOAT", T.NC_FLOAT), ("NC_SHORT", T.NC_SHORT),
                     ("NC_BYTE", T.NC_BYTE)):
        n = gib * GIB // T.xlen(xt)
        ms = timed(lambda: pncx.dev_fill(xt, buf, n))
        rows.append({"kernel": "pncx_dev_fill", "xtype": name, "bytes": gib * GIB, "ms": round(ms, 4),
                     "GBps": round(gib * GIB / ms / 1e6, 1), "frac_of_8TBps": round(gib * GIB / ms / 8e9, 4)})
    # one unaligned start: 3 bytes in, so the kernel's scalar head and tail run
    n = (gib * GIB - 16) // 8
    ms = timed(lambda: pncx.dev_fill(T.NC_DOUBLE, buf[3:], n))
    rows.append({"kernel": "pncx_dev_fill", "xtype": "NC_DOUBLE, start 3 B off", "bytes": n * 8, "ms": round(ms, 4),
                 "GBps": round(n * 8 / ms / 1e6, 1), "frac_of_8TBps": round(n * 8 / ms / 8e9, 4)})
    v = buf.view(torch.int64)
    ms = timed(lambda: v.fill_(-7))
    rows.append({"kernel": "torch fill_ (reference point)", "xtype": "int64", "bytes": gib * GIB, "ms": round(ms, 4),
                 "GBps": round(gib * GIB / ms / 1e6, 1), "frac_of_8TBps": round(gib * GIB / ms / 8e9, 4)})
    # spot check: the default NC_DOUBLE fill pattern, big-endian
    pncx.dev_fill(T.NC_DOUBLE, buf, 4)
    torch.cuda.synchronize()
    assert bytes(buf[:8].cpu().numpy()) == T.fill_bytes(T.NC_DOUBLE)[::-1]
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
