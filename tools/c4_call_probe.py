"""Where does the synchronous C4 call spend the time outside its kernel?
Wall-clock per pncx_dev_batch call (256 x 2^20 NC_SHORT/NC_FLOAT same-type
iputs, cached plan) with the library's kernel timing off and on, against the
async form queued back to back, and a 1-segment tiny batch (pure turnaround).

    python tools/c4_call_probe.py
"""
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    keep, segs = [], []
    fb = {x: (ctypes.c_uint8 * 16)(*T.fill_bytes(x)) for x in (T.NC_SHORT, T.NC_FLOAT)}
    for v in range(256):
        xt, it, isz = (T.NC_SHORT, T.ITYPE_SHORT, 2) if v % 2 == 0 else (T.NC_FLOAT, T.ITYPE_FLOAT, 4)
        ib = torch.empty((1 << 20) * isz // 8, dtype=torch.int64, device="cuda").random_()
        xb = torch.empty((1 << 20) * isz, dtype=torch.uint8, device="cuda")
        keep += [ib, xb]
        segs.append(pncx.Seg(T.PNCX_PUT, 5, xt, it, 1 << 20, xb.data_ptr(), ib.data_ptr(),
                             ctypes.cast(fb[xt], ctypes.c_void_p).value))
    big = (pncx.Seg * 256)(*segs)
    tiny_b = torch.empty(4096, dtype=torch.uint8, device="cuda")
    tiny = (pncx.Seg * 1)(pncx.Seg(T.PNCX_PUT, 5, T.NC_FLOAT, T.ITYPE_FLOAT, 512, tiny_b.data_ptr(),
                                   tiny_b.data_ptr() + 2048, ctypes.cast(fb[T.NC_FLOAT], ctypes.c_void_p).value))
    stv = (ctypes.c_int * 256)()
    dst = torch.zeros(256, dtype=torch.int32, device="cuda")
    dp = ctypes.c_void_p(dst.data_ptr())
    f_sync = lib.pncx_dev_batch
    f_async = lib.pncx_dev_batch_async

    def run(name, fn, n=200):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        per = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            per.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t0) * 1e6 / n
        print(json.dumps({"case": name, "median_us": round(statistics.median(per), 2),
                          "p10_us": round(sorted(per)[n // 10], 2), "loop_us_per_call": round(tot, 2)}), flush=True)

    run("tiny sync", lambda: f_sync(tiny, 1, stv, sp))
    run("tiny async", lambda: f_async(tiny, 1, dp, sp))
    run("nop ctypes", lambda: lib.pncx_xlen(5))
    run("c4 sync", lambda: f_sync(big, 256, stv, sp))
    lib.pncx_dev_batch_timing(1)
    run("c4 sync timed", lambda: f_sync(big, 256, stv, sp))
    tot, calls = ctypes.c_double(), ctypes.c_longlong()
    lib.pncx_dev_batch_kernel_ms(ctypes.byref(tot), ctypes.byref(calls))
    print(json.dumps({"case": "c4 kernel by lib events", "us": round(tot.value * 1e3 / calls.value, 2)}))
    lib.pncx_dev_batch_timing(0)
    run("c4 async", lambda: f_async(big, 256, dp, sp))


if __name__ == "__main__":
    main()
