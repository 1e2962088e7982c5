"""Rate of the varm transpose (k_imap_tile, NC_DOUBLE <- double put,
imap = Fortran order) over a list of shapes: which extents of the packed
fastest dimension P lose, and whether it is the 32-byte sector alignment
of the packed rows (P * 8 bytes).  Steady state: 10 launches between events.

    python tools/transpose_probe.py 1024x1024x250 1024x1024x252 ...
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    fb = np.frombuffer(T.fill_bytes(T.NC_DOUBLE) + b"\0" * 8, np.uint8).copy()
    fp = ctypes.c_void_p(fb.ctypes.data)
    gather = os.environ.get("PROBE_DIR", "put") == "put"
    for shape in sys.argv[1:]:
        cnt = [int(x) for x in shape.split("x")]
        imap = [1, cnt[0], cnt[0] * cnt[1]]
        n = cnt[0] * cnt[1] * cnt[2]
        u = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
        x = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
        c = np.asarray(cnt, np.int64)
        m = np.asarray(imap, np.int64)
        args = (5, T.NC_DOUBLE, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(u.data_ptr()), 3,
                ctypes.c_void_p(c.ctypes.data), ctypes.c_void_p(m.ctypes.data), T.ITYPE_DOUBLE)
        if gather:
            fn = lambda: lib.pncx_dev_putn_imap(*args, fp, ctypes.c_void_p(st.data_ptr()), sp)
        else:
            fn = lambda: lib.pncx_dev_getn_imap(*args, ctypes.c_void_p(st.data_ptr()), sp)
        fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
        for a, b in ev:
            a.record()
            for _ in range(10):
                fn()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)[3] / 10
        gbs = n * 16 / ms / 1e6
        print(json.dumps({"shape": shape, "dir": "put" if gather else "get", "row_bytes": cnt[2] * 8,
                          "row_mod32": cnt[2] * 8 % 32, "row_mod128": cnt[2] * 8 % 128, "ms": round(ms, 4),
                          "GB_per_s": round(gbs, 1), "frac": round(gbs / 8000, 4)}), flush=True)
        del u, x


if __name__ == "__main__":
    main()
