"""Does buffer placement explain C4's gap to a flat copy?  

The same C4 batch (256 variables x 2^20 elements, NC_SHORT / NC_FLOAT
alternating, same-type iput: one k_batch_swapmix launch) over four buffer
placements, in one process, interleaved round by round:
    torch_sep  one torch allocation per buffer (what bench.py does; torch's
               caching allocator carves 2/4 MiB blocks out of 20 MiB segments)
    hip_sep    one hipMalloc per buffer (512 separate allocations)
    pool       one 768 MiB allocation for the internal buffers and one for the
               external ones, variables back to back (sub-ranges)
    flat2      the same bytes as two segments (all NC_SHORT, all NC_FLOAT)
HIP events around every pncx_dev_batch_async launch on the launch stream.

    python tools/c4_placement.py [--rounds 8] [--reps 20] [--only NAME]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NVAR, NEL = 256, 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--steady", action="store_true",
                    help="time --reps launches back to back between two events instead of each launch alone")
    a = ap.parse_args()
    import torch
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    hip = ctypes.CDLL("libamdhip64.so")
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    fills = {}
    keep = []

    def fillp(xt):
        if xt not in fills:
            fills[xt] = (ctypes.c_uint8 * 16)(*T.fill_bytes(xt))
        return ctypes.cast(fills[xt], ctypes.c_void_p).value

    def kind(v):
        return (T.NC_SHORT, T.ITYPE_SHORT, 2) if v % 2 == 0 else (T.NC_FLOAT, T.ITYPE_FLOAT, 4)

    def seg(xt, it, n, xp, ip):
        return pncx.Seg(T.PNCX_PUT, 5, xt, it, n, xp, ip, fillp(xt))

    def hip_alloc(nbytes):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) == 0
        keep.append(p)
        return p.value

    def fill_bytes(ptr, nbytes, seed):
        t = torch.empty(nbytes // 8, dtype=torch.int64, device="cuda")
        t.random_(generator=torch.Generator(device="cuda").manual_seed(seed))
        assert hip.hipMemcpy(ctypes.c_void_p(ptr), ctypes.c_void_p(t.data_ptr()), ctypes.c_size_t(nbytes), 3) == 0

    layouts = {}
    # torch_sep
    segs = []
    for v in range(NVAR):
        xt, it, isz = kind(v)
        ib = torch.empty(NEL * isz // 8, dtype=torch.int64, device="cuda").random_()
        xb = torch.empty(NEL * isz, dtype=torch.uint8, device="cuda")
        keep += [ib, xb]
        segs.append(seg(xt, it, NEL, xb.data_ptr(), ib.data_ptr()))
    layouts["torch_sep"] = segs
    # hip_sep
    segs = []
    for v in range(NVAR):
        xt, it, isz = kind(v)
        ip, xp = hip_alloc(NEL * isz), hip_alloc(NEL * isz)
        fill_bytes(ip, NEL * isz, v)
        segs.append(seg(xt, it, NEL, xp, ip))
    layouts["hip_sep"] = segs
    # pool
    tot = NVAR // 2 * NEL * 6
    ipool = torch.empty(tot // 8, dtype=torch.int64, device="cuda").random_()
    xpool = torch.empty(tot, dtype=torch.uint8, device="cuda")
    keep += [ipool, xpool]
    segs, off = [], 0
    for v in range(NVAR):
        xt, it, isz = kind(v)
        segs.append(seg(xt, it, NEL, xpool.data_ptr() + off, ipool.data_ptr() + off))
        off += NEL * isz
    layouts["pool"] = segs
    # flat2
    h = NVAR // 2 * NEL
    layouts["flat2"] = [seg(T.NC_SHORT, T.ITYPE_SHORT, h, xpool.data_ptr(), ipool.data_ptr()),
                        seg(T.NC_FLOAT, T.ITYPE_FLOAT, h, xpool.data_ptr() + 2 * h, ipool.data_ptr() + 2 * h)]
    if a.only:
        layouts = {a.only: layouts[a.only]}
    arrs = {}
    for k, v in layouts.items():       # (plain stores were compared through a since-removed switch)
        arrs[(k, "nt_sc1")] = (pncx.Seg * len(v))(*v)
    dst = torch.zeros(NVAR, dtype=torch.int32, device="cuda")
    dp = ctypes.c_void_p(dst.data_ptr())
    moved = NVAR // 2 * NEL * (2 + 2 + 4 + 4)
    res = {k: [] for k in arrs}
    torch.cuda.synchronize()
    for r in range(a.rounds + 1):
        for (k, pol), arr in arrs.items():
            for _ in range(3):
                assert lib.pncx_dev_batch_async(arr, len(arr), dp, sp) == 0
            if a.steady:    # reps launches back to back between two events (the sweeps' method)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    assert lib.pncx_dev_batch_async(arr, len(arr), dp, sp) == 0
                e1.record(stream)
                torch.cuda.synchronize()
                if r > 0:
                    res[(k, pol)].append(e0.elapsed_time(e1) / a.reps)
                continue
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record(stream)
                assert lib.pncx_dev_batch_async(arr, len(arr), dp, sp) == 0
                e1.record(stream)
            torch.cuda.synchronize()
            if r > 0:
                res[(k, pol)] += [e0.elapsed_time(e1) for e0, e1 in ev]
    for k, v in res.items():
        med, best = statistics.median(v), min(v)
        print(json.dumps({"layout": k[0], "store": k[1], "median_ms": round(med, 4), "best_ms": round(best, 4),
                          "median_GBps": round(moved / med / 1e6, 1), "frac_median": round(moved / med / 8e9, 4),
                          "frac_best": round(moved / best / 8e9, 4), "launches": len(v)}), flush=True)


if __name__ == "__main__":
    main()
