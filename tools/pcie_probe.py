"""PCIe probe for the host-ended path: raw copy rates and staging variants."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    hip = ctypes.CDLL("libamdhip64.so.7")
    GB = 1e9
    nbytes = 4 << 30
    res = {}
    pin = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def t(fn, reps=3):
        fn(); torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter(); fn(); torch.cuda.synchronize(); best = min(best, time.perf_counter() - t0)
        return best
    res["h2d_pinned_GBps"] = nbytes / t(lambda: dev.copy_(pin, non_blocking=True)) / GB
    res["d2h_pinned_GBps"] = nbytes / t(lambda: pin.copy_(dev, non_blocking=True)) / GB
    half = nbytes // 2

    def both():
        with torch.cuda.stream(s1):
            dev[:half].copy_(pin[:half], non_blocking=True)
        with torch.cuda.stream(s2):
            pin[half:].copy_(dev[half:], non_blocking=True)
    res["h2d+d2h_concurrent_GBps_total"] = nbytes / t(both) / GB
    # hipHostRegister cost on a pageable buffer
    buf = np.frombuffer(np.random.default_rng(1).bytes(nbytes), np.uint8).copy()
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(nbytes), 0)
    res["hipHostRegister_4GiB_s"] = time.perf_counter() - t0
    res["hipHostRegister_rc"] = rc
    if rc == 0:
        n8 = nbytes // 8
        p = ctypes.c_void_p(buf.ctypes.data)
        res["in_swapn_registered_slab_GiBps"] = nbytes / t(lambda: lib.pncx_in_swapn(p, n8, 8)) / (1 << 30)
        t0 = time.perf_counter()
        hip.hipHostUnregister(ctypes.c_void_p(buf.ctypes.data))
        res["hipHostUnregister_s"] = time.perf_counter() - t0
    for k, v in list(res.items()):
        if isinstance(v, float):
            res[k] = round(v, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
