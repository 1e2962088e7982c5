"""HBM rate of the ncmpidiff first-difference kernel (pncx_dev_first_diff).

Worst case for the search: the arrays agree everywhere (or differ only within
tolerance), so both are streamed in full.  Algorithmic bytes per launch =
2 x n x sizeof(T) (read only).  Timed with HIP events on the launch stream;
the call includes the 8-byte result read-back and a stream sync.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from pnetcdf_amd import nctypes as T  # noqa: E402
from pnetcdf_amd import ncmpidiff  # noqa: E402

GIB = 1 << 30


def run(dtype, itype, gib, tol, td, tr, reps=10):
    n = int(gib * GIB) // torch.empty(0, dtype=dtype).element_size()
    a = torch.randn(n, dtype=torch.float64, device="cuda").mul_(1000).to(dtype)
    b = a.clone()
    if tol and dtype.is_floating_point:
        b.mul_(1 + 1e-7)                  # every element differs, all within the ratio tolerance
    st = torch.cuda.current_stream()
    for _ in range(2):
        assert ncmpidiff.first_diff(a, b, n, itype, tol, td, tr) == -1
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        ncmpidiff.first_diff(a, b, n, itype, tol, td, tr)
        e1.record(st)
    torch.cuda.synchronize()
    ms = sum(e0.elapsed_time(e1) for e0, e1 in ev) / reps
    nbytes = 2 * n * a.element_size()
    return {"dtype": str(dtype).replace("torch.", ""), "tolerance": bool(tol), "bytes_read": nbytes,
            "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1), "frac_of_8TBps": round(nbytes / ms / 8e9, 4)}


def main():
    torch.cuda.init()
    rows = [run(torch.float64, T.ITYPE_DOUBLE, 8, False, 0, 0),
            run(torch.float64, T.ITYPE_DOUBLE, 8, True, 0.0, 1e-3),
            run(torch.float32, T.ITYPE_FLOAT, 8, True, 0.0, 1e-3),
            run(torch.int16, T.ITYPE_SHORT, 8, False, 0, 0),
            run(torch.int32, T.ITYPE_INT, 8, True, 0.5, 0.0)]
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
