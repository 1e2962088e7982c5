"""Throughput of the device-resident conversion kernels over the (xtype,
itype) matrix (HIP events around each launch; algorithmic bytes = n *
(xsize + isize)).  Usage: python tools/matrix_bench.py [--n N] [--all]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 31)
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pairs", default="", help="comma list of dir:xtype:itype, e.g. get:float:ulonglong")
    ap.add_argument("--no-status", action="store_true", help="pass no status word (no NC_ERANGE tracking)")
    args = ap.parse_args()
    import torch
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    nmax = args.n
    xbuf = torch.empty(nmax * 8, dtype=torch.uint8, device="cuda")
    ibuf = torch.empty(nmax * 8, dtype=torch.uint8, device="cuda")
    xbuf.view(torch.int64).random_()
    ibuf.view(torch.int64).random_()
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    px, pi, ps = (ctypes.c_void_p(t.data_ptr()) for t in (xbuf, ibuf, st))
    if args.no_status:
        ps = None
    if args.pairs:
        pairs = []
        for tok in args.pairs.split(","):
            d, x, i = tok.split(":")
            pairs.append((T.PNCX_GET if d == "get" else T.PNCX_PUT, T.XTYPES[x], T.ITYPES[i]))
    elif args.all:
        pairs = [(d, x, i) for d in (T.PNCX_GET, T.PNCX_PUT) for x in T.NUMERIC_XTYPES for i in T.NUMERIC_ITYPES]
    else:
        pairs = [(T.PNCX_GET, T.NC_INT, T.ITYPE_DOUBLE), (T.PNCX_GET, T.NC_DOUBLE, T.ITYPE_DOUBLE),
                 (T.PNCX_GET, T.NC_SHORT, T.ITYPE_SHORT), (T.PNCX_GET, T.NC_FLOAT, T.ITYPE_FLOAT),
                 (T.PNCX_PUT, T.NC_SHORT, T.ITYPE_FLOAT), (T.PNCX_PUT, T.NC_FLOAT, T.ITYPE_DOUBLE),
                 (T.PNCX_GET, T.NC_BYTE, T.ITYPE_DOUBLE), (T.PNCX_PUT, T.NC_BYTE, T.ITYPE_DOUBLE),
                 (T.PNCX_GET, T.NC_SHORT, T.ITYPE_DOUBLE), (T.PNCX_PUT, T.NC_SHORT, T.ITYPE_LONGLONG),
                 (T.PNCX_GET, T.NC_UBYTE, T.ITYPE_INT), (T.PNCX_PUT, T.NC_UBYTE, T.ITYPE_FLOAT),
                 (T.PNCX_GET, T.NC_INT64, T.ITYPE_FLOAT), (T.PNCX_PUT, T.NC_INT, T.ITYPE_DOUBLE),
                 (T.PNCX_GET, T.NC_DOUBLE, T.ITYPE_FLOAT), (T.PNCX_GET, T.NC_FLOAT, T.ITYPE_DOUBLE)]
    res = []
    for d, x, i in pairs:
        # >= 4 GiB moved per launch so the 256 MiB Infinity Cache cannot serve it
        n = min(nmax, (4 << 30) // (T.xlen(x) + T.ilen(i)))
        fb = np.frombuffer(T.fill_bytes(x) + b"\0" * 8, np.uint8).copy()
        fp = ctypes.c_void_p(fb.ctypes.data)

        def run():
            if d == T.PNCX_GET:
                rc = lib.pncx_dev_getn(5, x, px, pi, n, i, ps, sp)
            else:
                rc = lib.pncx_dev_putn(5, x, px, pi, n, i, fp, ps, sp)
            assert rc == 0, rc
        run()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record()
            run()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)[args.reps // 2]
        by = n * (T.xlen(x) + T.ilen(i))
        r = {"dir": "get" if d == T.PNCX_GET else "put", "xtype": T.XNAME[x], "itype": T.INAME[i],
             "ms": round(ms, 4), "GBps": round(by / ms / 1e6, 1), "frac": round(by / ms / 1e6 / 8000, 4)}
        res.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
