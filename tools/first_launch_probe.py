"""What the first launch from each kernel file costs (HIP loads a file's code
object on a device at its first launch), without torch: libpncx alone,
ctypes, one process per ordering.  Prints ms per first call and a second
call of the same entry point for comparison.

    python tools/first_launch_probe.py [order]     order: letters s p g d
        s  pncx_dev_swapn (pncx_kern_swap.hip)   p  pncx_dev_putn NC_INT <- double (pncx_kern_put.hip, NC_INT object)
        g  pncx_dev_getn NC_INT -> double (pncx_kern_get.hip, NC_INT object)   d  pncx_dev_first_diff (pncx_kern_diff.hip)
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    order = sys.argv[1] if len(sys.argv) > 1 else "spgd"
    t0 = time.perf_counter()
    lib = ctypes.CDLL(os.environ.get("PNCX_LIB_PATH", os.path.join(ROOT, "pnetcdf_amd", "lib", "libpncx.so")))
    hip = ctypes.CDLL("libamdhip64.so")
    t_load = time.perf_counter() - t0
    t0 = time.perf_counter()
    n = ctypes.c_int()
    assert hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    t_init = time.perf_counter() - t0
    bufs = []
    for _ in range(4):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20)) == 0
        bufs.append(p)
    a, b, st, first = bufs
    assert hip.hipMemset(a, 0, ctypes.c_size_t(1 << 20)) == 0 and hip.hipMemset(b, 0, ctypes.c_size_t(1 << 20)) == 0
    fill = (ctypes.c_uint8 * 16)()
    NC_INT, ITYPE_DOUBLE = 4, 9

    calls = {
        "s": lambda: lib.pncx_dev_swapn(b, a, ctypes.c_longlong(1024), 4, None),
        "p": lambda: lib.pncx_dev_putn(5, NC_INT, b, a, ctypes.c_longlong(1024), ITYPE_DOUBLE, fill, st, None),
        "g": lambda: lib.pncx_dev_getn(5, NC_INT, a, b, ctypes.c_longlong(1024), ITYPE_DOUBLE, st, None),
        "d": lambda: lib.pncx_dev_first_diff(a, b, ctypes.c_longlong(1024), ITYPE_DOUBLE, 0, ctypes.c_double(0),
                                             ctypes.c_double(0), first, None),
    }
    out = {"load_ms": round(t_load * 1e3, 2), "hip_init_ms": round(t_init * 1e3, 2)}
    for k in order:
        for rep in ("first", "second"):
            t0 = time.perf_counter()
            rc = calls[k]()
            assert hip.hipDeviceSynchronize() == 0
            out[f"{k}_{rep}_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
            out[f"{k}_rc"] = rc
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
