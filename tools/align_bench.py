"""Rate of the streaming kernels on buffers whose start is not line-aligned:
in-place 8-byte swap (C2 kernel) and NC_INT -> double (C3 kernel), 8 GiB
moved-scale buffers at byte offsets 0 / 8 / 16 / 64 from a 256-byte
aligned allocation.  HIP events, median of 10."""
import ctypes
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
    L = pncx.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    buf = torch.empty(4 * GIB + 4096, dtype=torch.uint8, device="cuda")
    out = torch.empty(8 * GIB + 4096, dtype=torch.uint8, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    for off in (0, 8, 16, 64):
        n = 4 * GIB // 8
        p = ctypes.c_void_p(buf.data_ptr() + off)
        ms = timed(lambda: L.pncx_dev_in_swapn(p, ctypes.c_longlong(n), 8, sp))
        print(json.dumps({"kernel": "in_swapn 8B", "offset": off, "GBps": round(16 * n / ms / 1e6, 1)}), flush=True)
        n = 2 * GIB // 4
        px, pi = ctypes.c_void_p(buf.data_ptr() + off), ctypes.c_void_p(out.data_ptr() + 2 * off)
        ms = timed(lambda: L.pncx_dev_getn(5, T.NC_INT, px, pi, ctypes.c_longlong(n), T.ITYPE_DOUBLE,
                                           ctypes.c_void_p(st.data_ptr()), sp))
        print(json.dumps({"kernel": "getn NC_INT->double", "offset": off, "GBps": round(12 * n / ms / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
