"""C4 against the flat swap of the same bytes, for PMC passes (VERDICT r04
weak #5: "the loss is ramp/drain and placement; no counter separates the
two").  One mode per process, `--reps` launches back to back:
    batch  the bench's C4: 256 variables x 2^20 elements, NC_SHORT / NC_FLOAT
           alternating, one torch allocation per buffer, one
           pncx_dev_batch_async launch (k_batch_swapmix)
    flat2  the same bytes as two segments of one pool through the same
           batch kernel (placement and per-variable boundaries removed)
    flat   the same 768 MiB pair as one NC_FLOAT swap, pncx_dev_putn
           (k_tile<SwapOp<4>>, the flat ceiling)
Prints the median launch time (HIP events on the launch stream).

    python tools/c4_pmc_probe.py MODE [--reps 20]
    rocprofv3 --pmc ... --kernel-trace -- python3 tools/c4_pmc_probe.py MODE
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
    ap.add_argument("mode", choices=["batch", "flat2", "flat"])
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    fills = {xt: (ctypes.c_uint8 * 16)(*T.fill_bytes(xt)) for xt in (T.NC_SHORT, T.NC_FLOAT)}
    keep = []

    def fillp(xt):
        return ctypes.cast(fills[xt], ctypes.c_void_p).value

    def seg(xt, it, n, xp, ip):
        return pncx.Seg(T.PNCX_PUT, 5, xt, it, n, xp, ip, fillp(xt))

    tot = NVAR // 2 * NEL * 6                      # 768 MiB per side
    dst = torch.zeros(NVAR, dtype=torch.int32, device="cuda")
    dp = ctypes.c_void_p(dst.data_ptr())
    if a.mode == "batch":
        segs = []
        for v in range(NVAR):
            xt, it, isz = (T.NC_SHORT, T.ITYPE_SHORT, 2) if v % 2 == 0 else (T.NC_FLOAT, T.ITYPE_FLOAT, 4)
            ib = torch.empty(NEL * isz // 8, dtype=torch.int64, device="cuda").random_()
            xb = torch.empty(NEL * isz, dtype=torch.uint8, device="cuda")
            keep += [ib, xb]
            segs.append(seg(xt, it, NEL, xb.data_ptr(), ib.data_ptr()))
    else:
        ipool = torch.empty(tot // 8, dtype=torch.int64, device="cuda").random_()
        xpool = torch.empty(tot, dtype=torch.uint8, device="cuda")
        keep += [ipool, xpool]
        h = NVAR // 2 * NEL
        segs = [seg(T.NC_SHORT, T.ITYPE_SHORT, h, xpool.data_ptr(), ipool.data_ptr()),
                seg(T.NC_FLOAT, T.ITYPE_FLOAT, h, xpool.data_ptr() + 2 * h, ipool.data_ptr() + 2 * h)]
    arr = (pncx.Seg * len(segs))(*segs)
    st = torch.zeros(1, dtype=torch.int32, device="cuda")

    def launch():
        if a.mode == "flat":
            assert lib.pncx_dev_putn(5, T.NC_FLOAT, ctypes.c_void_p(xpool.data_ptr()),
                                     ctypes.c_void_p(ipool.data_ptr()), tot // 4, T.ITYPE_FLOAT,
                                     ctypes.c_void_p(fillp(T.NC_FLOAT)), ctypes.c_void_p(st.data_ptr()), sp) == 0
        else:
            assert lib.pncx_dev_batch_async(arr, len(arr), dp, sp) == 0

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    for e0, e1 in ev:
        e0.record(stream)
        launch()
        e1.record(stream)
    torch.cuda.synchronize()
    ms = statistics.median(e0.elapsed_time(e1) for e0, e1 in ev)
    moved = 2 * tot
    print(json.dumps({"mode": a.mode, "median_ms": round(ms, 4), "GBps": round(moved / ms / 1e6, 1),
                      "frac": round(moved / ms / 8e9, 4), "launches": a.reps}), flush=True)


if __name__ == "__main__":
    main()
