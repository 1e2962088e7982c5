"""Tile skew sweep for the transposes whose packed column stride lies just
under a multiple of 2 MiB (the DRAM-bank conflicts of x254).
Round 4 tried skews 0, 1 (diagonal), 8 and 32 and ships 8 (put) / 32 (get)
for that stride class; this sweeps the values between, in one process, the
skews interleaved round by round (PNCX_XPOSE_ORDER=k: tile p0 shifted by k
tiles per u tile; -1 = the shipped choice).  NC_DOUBLE <- double, imap in
Fortran order, 10 launches between events, median of 5.

    python tools/xpose_skew_sweep.py [--rounds 2] [--ks -1,2,3,4,...]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = ["1024x1024x254", "1024x1x260096"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--ks", default="-1,2,3,4,5,6,8,12,16,24,32,48,64")
    a = ap.parse_args()
    ks = [int(k) for k in a.ks.split(",")]
    import torch
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    fb = np.frombuffer(T.fill_bytes(T.NC_DOUBLE) + b"\0" * 8, np.uint8).copy()
    fp = ctypes.c_void_p(fb.ctypes.data)
    res = {}
    for shape in SHAPES:
        cnt = [int(x) for x in shape.split("x")]
        imap = [1, cnt[0], cnt[0] * cnt[1]]
        n = cnt[0] * cnt[1] * cnt[2]
        u = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
        x = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
        c = np.asarray(cnt, np.int64)
        m = np.asarray(imap, np.int64)
        args = (5, T.NC_DOUBLE, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(u.data_ptr()), 3,
                ctypes.c_void_p(c.ctypes.data), ctypes.c_void_p(m.ctypes.data), T.ITYPE_DOUBLE)
        fns = {"put": lambda: lib.pncx_dev_putn_imap(*args, fp, ctypes.c_void_p(st.data_ptr()), sp),
               "get": lambda: lib.pncx_dev_getn_imap(*args, ctypes.c_void_p(st.data_ptr()), sp)}
        for r in range(a.rounds):
            order = ks if r % 2 == 0 else ks[::-1]
            for d, fn in fns.items():
                for k in order:
                    pncx.knob_set("XPOSE_ORDER", k)
                    fn()
                    torch.cuda.synchronize()
                    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                          for _ in range(5)]
                    for e0, e1 in ev:
                        e0.record()
                        for _ in range(10):
                            fn()
                        e1.record()
                    torch.cuda.synchronize()
                    ms = statistics.median(e0.elapsed_time(e1) for e0, e1 in ev) / 10
                    res.setdefault((shape, d, k), []).append(round(n * 16 / ms / 8e9, 4))
        pncx.knob_set("XPOSE_ORDER", -1)
        del u, x
    for (shape, d, k), v in sorted(res.items()):
        print(json.dumps({"shape": shape, "dir": d, "skew": k, "frac": v}), flush=True)


if __name__ == "__main__":
    main()
