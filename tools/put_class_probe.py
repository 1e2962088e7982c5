"""Is the C4 secondary variant's float -> NC_SHORT batch class (k_batch<PutOp>,
75-76 % of peak) slow because of its size or because it is a batch?

The same 128 x 2^20 float values (uniform in [-40000, 40000], ~18 % out of
range) converted to NC_SHORT as one flat pncx_dev_putn over one buffer pair
(k_tile) and as a pncx_dev_batch_async of 128 segments over 128 buffer pairs
(k_batch + the flag reduce), interleaved, 20 launches back to back between
two events per sample.  Algorithmic bytes: 6 per element.

    python tools/put_class_probe.py [--rounds 6]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    nvar, nel = 128, 1 << 20
    n = nvar * nel
    flat_i = torch.empty(n, dtype=torch.float32, device="cuda")
    bench.splitmix_uniform(torch, flat_i, 0x5EED0004, -40000.0, 40000.0)
    flat_x = torch.empty(n * 2, dtype=torch.uint8, device="cuda")
    fill = np.frombuffer(T.fill_bytes(T.NC_SHORT) + b"\0" * 8, np.uint8).copy()
    fst = torch.zeros(1, dtype=torch.int32, device="cuda")
    ins, outs, segs = [], [], []
    for v in range(nvar):
        ib = flat_i[v * nel:(v + 1) * nel].clone()
        xb = torch.empty(nel * 2, dtype=torch.uint8, device="cuda")
        ins.append(ib)
        outs.append(xb)
        segs.append(pncx.Seg(T.PNCX_PUT, 5, T.NC_SHORT, T.ITYPE_FLOAT, nel, xb.data_ptr(), ib.data_ptr(),
                             fill.ctypes.data))
    arr = (pncx.Seg * nvar)(*segs)
    dst = torch.zeros(nvar, dtype=torch.int32, device="cuda")
    dp = ctypes.c_void_p(dst.data_ptr())

    def flat():
        assert lib.pncx_dev_putn(5, T.NC_SHORT, ctypes.c_void_p(flat_x.data_ptr()),
                                 ctypes.c_void_p(flat_i.data_ptr()), n, T.ITYPE_FLOAT,
                                 ctypes.c_void_p(fill.ctypes.data), ctypes.c_void_p(fst.data_ptr()), sp) == 0

    def batch():
        assert lib.pncx_dev_batch_async(arr, nvar, dp, sp) == 0

    res = {"flat": [], "batch": []}
    for r in range(a.rounds + 1):
        for name, f in (("flat", flat), ("batch", batch)):
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                f()
            e1.record(stream)
            torch.cuda.synchronize()
            if r > 0:
                res[name].append(e0.elapsed_time(e1) / a.reps)
    same = all(torch.equal(outs[v], flat_x[v * nel * 2:(v + 1) * nel * 2]) for v in range(nvar))
    for k, v in res.items():
        med = statistics.median(v)
        print(json.dumps({"form": k, "median_ms": round(med, 4), "frac": round(6 * n / (med * 1e-3) / 8e12, 4),
                          "all": [round(x, 4) for x in v], "outputs_equal": same}), flush=True)


if __name__ == "__main__":
    main()
