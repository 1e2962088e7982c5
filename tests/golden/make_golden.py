"""Generate tests/golden/edge_vectors.npz from the pinned CPU oracle.

For every (xtype, itype) of the conversion matrix (10 x 11) and both
directions, a fixed list of edge inputs (type MIN/MAX, MIN-1/MAX+1, +-0,
+-inf, quiet/signalling NaN with payloads, denormals, 2^31/2^32/2^63/2^64
boundaries, f64->f32 rounding ties, FLT_MAX +- 1/2 ulp) is converted by the
oracle with the default fill and with a user fill, recording output bytes
and status.  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402
from pnetcdf_amd import nctypes as T  # noqa: E402

INT_EDGES = [0, 1, -1, 2, -2, 5, 100, 126, 127, 128, 129, -127, -128, -129, -130, 254, 255, 256, 257,
             32766, 32767, 32768, 32769, -32767, -32768, -32769, 65534, 65535, 65536, 65537,
             2**31 - 2, 2**31 - 1, 2**31, 2**31 + 1, -2**31 + 1, -2**31, -2**31 - 1,
             2**32 - 2, 2**32 - 1, 2**32, 2**32 + 1, 2**53 - 1, 2**53, 2**53 + 1, 2**53 + 3,
             2**24 - 1, 2**24, 2**24 + 1, 2**24 + 3, 2**62, 2**63 - 2, 2**63 - 1, -2**63 + 1, -2**63,
             2**63, 2**63 + 1, 2**64 - 1025, 2**64 - 2, 2**64 - 1, 0x5555555555555555, -0x7ffffffffffffc01,
             (1 << 63) | 1023, 0x7fffffffffffffff - 512]


def float_edges():
    f = np.float64
    v = [0.0, -0.0, 0.5, -0.5, 0.49999999999999994, 1.0, -1.0, 1.5, -1.5, 2.5, -2.5, 126.9, 127.0, 127.5,
         127.99999, 128.0, -128.0, -128.5, -128.99999, -129.0, 254.5, 255.0, 255.5, 256.0, -0.9, -1e-300,
         32767.0, 32767.5, 32767.9, 32768.0, -32768.0, -32768.5, -32769.0, 65535.0, 65535.5, 65536.0,
         2147483647.0, 2147483647.5, 2147483648.0, -2147483648.0, -2147483648.5, -2147483649.0,
         4294967295.0, 4294967295.5, 4294967296.0, 9.223372036854775e18, 9.223372036854775808e18,
         -9.223372036854775808e18, 9.2233720368547758e18 * 1.0000000000000002, -9.223372036854777e18,
         1.8446744073709550e19, 1.8446744073709551616e19, 1.8446744073709555e19, 3.0e19,
         float(np.finfo(np.float32).max), float(np.finfo(np.float32).max) * (1 + 2 ** -25),
         float(np.nextafter(np.float64(np.finfo(np.float32).max), np.inf)),
         3.4028235677973366e+38, 3.4028235677973362e+38, 3.4028236e38, -3.4028236e38,
         float(np.finfo(np.float64).max), -float(np.finfo(np.float64).max), float("inf"), float("-inf"),
         1e-45, 1.4e-45, 7e-46, 1e-40, -1e-40, 1.1754943508222875e-38, 5e-324, -5e-324, 2.2250738585072014e-308,
         1.0 + 2 ** -24, 1.0 + 3 * 2 ** -24, 1.0 + 2 ** -23 + 2 ** -24, 16777217.0, 16777219.0,
         9.9692099683868690e+36, 1e10, -3.7, 1e300, -1e300, 0.1, 1.0 / 3.0]
    v = [f(x) for x in v]
    bits = [0x7ff8000000000000, 0xfff8000000000000, 0x7ff0000000000001, 0x7ff4000000000000,
            0xfff0000000000123, 0x7ff80000deadbeef, 0x7fffffffffffffff, 0x7ff0000020000000]
    v += [np.array([b], np.uint64).view(np.float64)[0] for b in bits]
    return np.array(v, np.float64)


def float32_edges():
    v = float_edges().astype(np.float32)
    bits = [0x7fc00000, 0xffc00000, 0x7f800001, 0x7fa00000, 0xff800123, 0x7fc0beef, 0x7fffffff,
            0x00000001, 0x80000001, 0x007fffff, 0x00800000]
    return np.concatenate([v, np.array(bits, np.uint32).view(np.float32)])


def edges_for(np_dtype):
    dt = np.dtype(np_dtype)
    if dt == np.float64:
        return float_edges()
    if dt == np.float32:
        return float32_edges()
    info = np.iinfo(dt)
    vals = [x for x in INT_EDGES if info.min <= x <= info.max] + [info.min, info.max, info.min + 1, info.max - 1]
    return np.array(vals, dtype=dt)


def main():
    out = {}
    rng = np.random.default_rng(0x5EED0000)
    for xt in T.NUMERIC_XTYPES:
        for it in T.NUMERIC_ITYPES:
            key = f"{T.XNAME[xt]}_{T.INAME[it]}"
            for cdf in (5, 2) if xt == T.NC_BYTE and it == T.ITYPE_UCHAR else (5,):
                k = key + ("_cdf2" if cdf == 2 else "")
                # GET: edges of the external type, stored big-endian
                xin = edges_for(T.XTYPE_NP[xt]).astype(T.XTYPE_BE[xt]).tobytes()
                res, st = O.getn(cdf, xt, xin, it)
                out[f"get_{k}_in"] = np.frombuffer(xin, np.uint8)
                out[f"get_{k}_out"] = np.frombuffer(res.tobytes(), np.uint8)
                out[f"get_{k}_st"] = np.array([st], np.int32)
                # PUT: edges of the internal type; default fill, user fill, NULL
                iin = edges_for(T.ITYPE_NP[it])
                n = iin.size
                xinit = rng.integers(0, 256, n * T.xlen(xt), dtype=np.uint8).tobytes()
                out[f"put_{k}_in"] = np.frombuffer(iin.tobytes(), np.uint8)
                out[f"put_{k}_xinit"] = np.frombuffer(xinit, np.uint8)
                for tag, fill in (("dflt", T.fill_bytes(xt)), ("user", T.fill_bytes(xt, 99)), ("null", None)):
                    xb, st = O.putn(cdf, xt, iin, it, fill=fill, xinit=xinit)
                    out[f"put_{k}_{tag}_out"] = np.frombuffer(xb, np.uint8)
                    out[f"put_{k}_{tag}_st"] = np.array([st], np.int32)
    np.savez_compressed(os.path.join(HERE, "edge_vectors.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
