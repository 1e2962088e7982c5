"""Host-buffer (PCIe-inclusive) rates of the drop-in entry points, next to
the CPU oracle on the same buffer.  The reference's path starts and ends in
host memory (user array <-> MPI-IO buffer); pncx_in_swapn / pncx_getn stage
through HBM in chunks over two HIP streams.

    python tools/host_roundtrip.py [--gib G]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, reps=5):
    """median of `reps` timed calls after one warm call"""
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    args = ap.parse_args()
    import torch  # noqa: F401  (shared HIP runtime)
    from oracle import oracle as O
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    GIB = float(1 << 30)
    nbytes = int(args.gib * GIB)
    n8 = nbytes // 8
    buf = np.frombuffer(np.random.default_rng(2).bytes(nbytes), np.uint64).copy()
    res = {"slab_gib": args.gib}
    p = ctypes.c_void_p(buf.ctypes.data)
    t = timeit(lambda: lib.pncx_in_swapn(p, n8, 8))
    res["in_swapn8_host_pageable"] = {"s": t, "slab_GiBps": nbytes / t / GIB, "moved_GiBps": 2 * nbytes / t / GIB}
    # pinned user buffer (what an application with hipHostMalloc'd buffers sees)
    pin = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    pp = ctypes.c_void_p(pin.data_ptr())
    t = timeit(lambda: lib.pncx_in_swapn(pp, n8, 8))
    res["in_swapn8_host_pinned"] = {"s": t, "slab_GiBps": nbytes / t / GIB, "moved_GiBps": 2 * nbytes / t / GIB}
    # pageable buffer registered once by the application (pncx_host_register)
    pncx.host_register(buf)
    t = timeit(lambda: lib.pncx_in_swapn(p, n8, 8))
    res["in_swapn8_host_registered"] = {"s": t, "slab_GiBps": nbytes / t / GIB, "moved_GiBps": 2 * nbytes / t / GIB}
    pncx.host_unregister(buf)
    # config-3 shape from host buffers: NC_INT -> double
    n4 = nbytes // 8          # ints (xbuf = nbytes/2, ibuf = nbytes)
    xb = np.frombuffer(np.random.default_rng(3).bytes(n4 * 4), np.uint8).copy()
    ib = np.empty(n4, np.float64)
    t = timeit(lambda: lib.pncx_getn(5, T.NC_INT, ctypes.c_void_p(xb.ctypes.data), ctypes.c_void_p(ib.ctypes.data),
                                     n4, T.ITYPE_DOUBLE))
    res["getn_int_double_host"] = {"s": t, "moved_GiBps": 12 * n4 / t / GIB}
    pncx.host_register(xb)
    pncx.host_register(ib)
    t = timeit(lambda: lib.pncx_getn(5, T.NC_INT, ctypes.c_void_p(xb.ctypes.data), ctypes.c_void_p(ib.ctypes.data),
                                     n4, T.ITYPE_DOUBLE))
    res["getn_int_double_host_registered"] = {"s": t, "moved_GiBps": 12 * n4 / t / GIB}
    pncx.host_unregister(xb)
    pncx.host_unregister(ib)
    # CPU oracle, 1 thread, same buffers
    t = timeit(lambda: O.lib().orc_in_swapn(p, n8, 8), reps=2)
    res["cpu_oracle_in_swapn8_1core"] = {"s": t, "moved_GiBps": 2 * nbytes / t / GIB}
    t = timeit(lambda: O.lib().orc_getn(5, T.NC_INT, ctypes.c_void_p(xb.ctypes.data), ctypes.c_void_p(ib.ctypes.data),
                                        n4, T.ITYPE_DOUBLE), reps=2)
    res["cpu_oracle_getn_int_double_1core"] = {"s": t, "moved_GiBps": 12 * n4 / t / GIB}
    for k, v in res.items():
        if isinstance(v, dict):
            v.update({kk: round(vv, 3) for kk, vv in v.items()})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
