"""File-level rates of the drop-in path (BASELINE.json configs[0] and the
file-level shape of configs[2]/[3]) on tmpfs, next to the reference's CPU
sequence restated with the oracle.

Our path:   pncx_nc_put_varm / get_varm  (GPU conversion, pwrite/pread)
            pncx_nc_iput_varm x N + wait_all (one batched conversion)
Reference:  put_vara_int_all of a same-type variable = in-place swap of the
            user buffer, write, swap back (ncmpio_getput.m4:186-214,269-270);
            get = read + swap (ncmpio_getput.m4:415-466, ncmpio_util.c:884-888);
            cross-type = per-request getn/putn into an xbuf (ncmpio_util.c:716-765).
            Restated here with oracle/pncx_oracle.c (gcc -O2, 1 thread) and
            POSIX pwrite/pread -- the reference library itself is not
            buildable here.

    python tools/file_bench.py [--dir /dev/shm] [--reps 5]
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
GIB = float(1 << 30)


def med(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/dev/shm")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--big-gib", type=float, default=1.0)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime)
    from oracle import oracle as O
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import ncfile as N
    OL = O.lib()
    res = {"dir": args.dir, "reps": args.reps}
    path = os.path.join(args.dir, f"pncx_bench_{os.getpid()}.nc")

    def ours_put_get(nel, xt, it, label):
        """NC_INT variable from an int buffer (full int32 range, edge values first)"""
        rng = np.random.default_rng(0x5EED0001)
        buf = rng.integers(-2**31, 2**31 - 1, nel, dtype=np.int64).astype(np.int32)
        buf[:4] = [-2**31, 2**31 - 1, 0, -1]
        err, ncid = N.create(path, N.NC_64BIT_DATA)
        N.def_dim(ncid, "x", nel)
        N.def_var(ncid, "v", xt, [0])
        assert N.enddef(ncid) == 0
        out = np.empty_like(buf)
        tp = med(lambda: N.put_var(ncid, 0, buf, [0], [nel]), args.reps)
        tg = med(lambda: N.get_var(ncid, 0, out, [0], [nel]), args.reps)
        assert N.close(ncid) == 0
        assert np.array_equal(out, buf), label
        xs = T.xlen(xt)
        os.unlink(path)
        return {"elements": nel, "external_bytes": nel * xs,
                "put_s": tp, "get_s": tg,
                "put_GiBps_external": nel * xs / tp / GIB, "get_GiBps_external": nel * xs / tg / GIB}

    def ref_cpu_same_type(nel, esize):
        """restated reference sequence for a same-type variable, one thread"""
        rng = np.random.default_rng(0x5EED0001)
        buf = np.frombuffer(rng.bytes(nel * esize), np.uint8).copy()
        fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
        p = ctypes.c_void_p(buf.ctypes.data)

        def put():
            OL.orc_in_swapn(p, nel, esize)            # ncmpio_getput.m4:211
            os.pwrite(fd, buf, 512)
            OL.orc_in_swapn(p, nel, esize)            # swap back, :270

        def get():
            data = os.pread(fd, nel * esize, 512)
            x = np.frombuffer(data, np.uint8).copy()
            OL.orc_in_swapn(ctypes.c_void_p(x.ctypes.data), nel, esize)
            return x
        tp = med(put, args.reps)
        tg = med(get, args.reps)
        os.close(fd)
        os.unlink(path)
        return {"put_s": tp, "get_s": tg, "put_GiBps_external": nel * esize / tp / GIB,
                "get_GiBps_external": nel * esize / tg / GIB, "threads": 1}

    # C1: 1-D 1M NC_INT, int buffer
    res["C1_ours"] = ours_put_get(1 << 20, T.NC_INT, T.ITYPE_INT, "c1")
    res["C1_reference_cpu_restated"] = ref_cpu_same_type(1 << 20, 4)
    # same shape, larger: where the GPU path amortises its launch/copy latency
    nbig = int(args.big_gib * GIB) // 4
    res["INT_big_ours"] = ours_put_get(nbig, T.NC_INT, T.ITYPE_INT, "big")
    res["INT_big_reference_cpu_restated"] = ref_cpu_same_type(nbig, 4)
    # config-3 shape at file level: NC_INT read as double
    err, ncid = N.create(path, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", nbig)
    N.def_var(ncid, "v", T.NC_INT, [0])
    N.enddef(ncid)
    src = np.random.default_rng(3).integers(-2**31, 2**31 - 1, nbig, dtype=np.int64).astype(np.int32)
    N.put_var(ncid, 0, src)
    out = np.empty(nbig, np.float64)
    tg = med(lambda: N.get_var(ncid, 0, out), args.reps)
    assert np.array_equal(out, src.astype(np.float64))
    N.close(ncid)
    raw = np.fromfile(path, np.uint8)[512:512 + nbig * 4].copy()
    outc = np.empty(nbig, np.float64)

    def ref_get_double():
        data = np.fromfile(path, np.uint8, count=512 + nbig * 4)[512:]
        OL.orc_getn(5, T.NC_INT, ctypes.c_void_p(data.ctypes.data), ctypes.c_void_p(outc.ctypes.data),
                    nbig, T.ITYPE_DOUBLE)
    tr = med(ref_get_double, args.reps)
    assert np.array_equal(outc, out)
    del raw
    os.unlink(path)
    res["C3_file_get_vara_double"] = {"elements": nbig, "ours_s": tg, "reference_cpu_restated_s": tr,
                                      "ours_GiBps_external": nbig * 4 / tg / GIB,
                                      "reference_GiBps_external": nbig * 4 / tr / GIB}
    # config-4 shape at file level: 256 x 2^20 iput (short/float) + wait_all
    nvar, nel = 256, 1 << 20
    err, ncid = N.create(path, N.NC_64BIT_DATA)
    N.def_dim(ncid, "x", nel)
    for v in range(nvar):
        N.def_var(ncid, f"v{v}", T.NC_SHORT if v % 2 == 0 else T.NC_FLOAT, [0])
    N.enddef(ncid)
    rng = np.random.default_rng(0x5EED0004)
    bufs = [rng.integers(-32768, 32767, nel, dtype=np.int16) if v % 2 == 0 else
            rng.standard_normal(nel).astype(np.float32) for v in range(nvar)]

    def ours_c4():
        reqs = [N.iput_var(ncid, v, bufs[v], [0], [nel])[1] for v in range(nvar)]
        err, st = N.wait_all(ncid, reqs)
        assert err == 0
    t4 = med(ours_c4, args.reps)
    N.close(ncid)
    ext = sum(b.nbytes for b in bufs)
    offs = []
    err, ncid = N.open(path)
    for v in range(nvar):
        offs.append(N.inq_varoffset(ncid, v)[1])
    N.close(ncid)
    fd = os.open(path, os.O_RDWR)

    def ref_c4():
        # per-request: in-place swap of the user buffer, write, swap back
        for v in range(nvar):
            b = bufs[v]
            OL.orc_in_swapn(ctypes.c_void_p(b.ctypes.data), nel, b.itemsize)
            os.pwrite(fd, b, offs[v])
            OL.orc_in_swapn(ctypes.c_void_p(b.ctypes.data), nel, b.itemsize)
    tr4 = med(ref_c4, args.reps)
    os.close(fd)
    os.unlink(path)
    res["C4_file_iput_wait_all"] = {"variables": nvar, "elements_per_var": nel, "ours_s": t4,
                                    "reference_cpu_restated_s": tr4, "ours_GiBps_external": ext / t4 / GIB,
                                    "reference_GiBps_external": ext / tr4 / GIB}
    for k, v in res.items():
        if isinstance(v, dict):
            for kk, vv in v.items():
                if isinstance(vv, float):
                    v[kk] = round(vv, 5)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
