"""Throughput of the fused pack+convert kernels (derived buftypes, varm) against
the contiguous kernel on the same element count.  Device-resident; HIP events
around 10 back-to-back launches; algorithmic bytes = n * (xsize + isize) (the gaps between
runs are not counted).

Workloads (NC_DOUBLE external <- double user buffer, put direction):
  halo3d    interior 254^3 of a 256^3 local array (ghost cells dropped): a 3-D
            subarray buftype, 64516 runs of 254 elements -> general table
  halo3d_varm  the same interior as a varm request (imap {L*L, L, 1})
  vector2   every other element (MPI_Type_vector(n, 1, 2)) -> uniform runs
  vector64  runs of 64 every 80 -> uniform runs
  vector256 runs of 256 every 272 -> uniform runs, one wave per run
  transpose varm with imap = Fortran order over a 512 x 512 x 128 request
  contig    plain pncx_dev_putn on the same n (the roofline reference)

    python tools/flex_bench.py [--reps 10]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--big", action="store_true",
                    help="every workload at >= 4 GiB moved per launch (2^28 elements and more)")
    ap.add_argument("--short-only", action="store_true",
                    help="only the short-run workloads (map widths, put and get)")
    args = ap.parse_args()
    big = args.big
    import torch
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    fb = np.frombuffer(T.fill_bytes(T.NC_DOUBLE) + b"\0" * 8, np.uint8).copy()
    fp = ctypes.c_void_p(fb.ctypes.data)

    def offs(v):
        a = np.ascontiguousarray(np.asarray(v, np.int64))
        return a, ctypes.c_void_p(a.ctypes.data)

    def timeit(fn, n):
        fn()
        torch.cuda.synchronize()
        # steady state: 10 launches of the same kernel between the events (a
        # single launch after a different kernel moved results by ~10 points
        # at these sizes, which are about the Infinity Cache's)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record()
            for _ in range(10):
                fn()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)[len(ev) // 2] / 10
        return ms, n * 16 / ms / 1e6

    res = []
    if args.short_only:
        short_runs(args, big, torch, T, pncx, lib, st, sp, fp, offs, timeit, res)
        report(res)
        return
    # halo3d: 256^3 local array, interior 254^3 (--big: 648^3, interior 646^3)
    L, I = (648, 646) if big else (256, 254)
    ub = torch.empty(L ** 3 * 8, dtype=torch.uint8, device="cuda")
    ub.view(torch.float64).normal_()
    z, y = np.meshgrid(np.arange(I), np.arange(I), indexing="ij")
    disp = (((z + 1) * L * L + (y + 1) * L + 1) * 8).reshape(-1)
    dt = pncx.DType(T.ITYPE_DOUBLE, disp.tolist(), [I] * disp.size, L ** 3 * 8)
    n = I ** 3
    xb = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
    c, cp = offs([n])
    res.append(("halo3d", dt.inq()["layout"], n) + timeit(
        lambda: lib.pncx_dev_putn_flex(5, T.NC_DOUBLE, ctypes.c_void_p(xb.data_ptr()), ctypes.c_void_p(ub.data_ptr()),
                                       1, cp, None, 1, dt.handle, fp, ctypes.c_void_p(st.data_ptr()), sp), n))
    # the same interior through varm (imap {L*L, L, 1} from the first interior element)
    cv, cvp = offs([I, I, I])
    iv, ivp = offs([L * L, L, 1])
    first = ((L * L + L + 1) * 8)
    res.append(("halo3d_varm", -1, n) + timeit(
        lambda: lib.pncx_dev_putn_imap(5, T.NC_DOUBLE, ctypes.c_void_p(xb.data_ptr()),
                                       ctypes.c_void_p(ub.data_ptr() + first), 3, cvp, ivp, T.ITYPE_DOUBLE, fp,
                                       ctypes.c_void_p(st.data_ptr()), sp), n))
    res.append(("contig", -1, n) + timeit(
        lambda: lib.pncx_dev_putn(5, T.NC_DOUBLE, ctypes.c_void_p(xb.data_ptr()), ctypes.c_void_p(ub.data_ptr()), n,
                                  T.ITYPE_DOUBLE, fp, ctypes.c_void_p(st.data_ptr()), sp), n))
    # vector2 / vector64 over 2^27 elements (--big: 2^28)
    for name, blen, stride in (("vector2", 1, 2), ("vector64", 64, 80), ("vector256", 256, 272)):
        nb = (1 << (28 if big else 27)) // blen
        span = nb * stride * 8
        u2 = torch.empty(span, dtype=torch.uint8, device="cuda")
        dtv = pncx.DType(T.ITYPE_DOUBLE, (np.arange(nb, dtype=np.int64) * stride * 8).tolist(), [blen] * nb, span)
        n2 = nb * blen
        x2 = torch.empty(n2 * 8, dtype=torch.uint8, device="cuda")
        c2, cp2 = offs([n2])
        res.append((name, dtv.inq()["layout"], n2) + timeit(
            lambda: lib.pncx_dev_putn_flex(5, T.NC_DOUBLE, ctypes.c_void_p(x2.data_ptr()),
                                           ctypes.c_void_p(u2.data_ptr()), 1, cp2, None, 1, dtv.handle, fp,
                                           ctypes.c_void_p(st.data_ptr()), sp), n2))
        del u2, x2
    short_runs(args, big, torch, T, pncx, lib, st, sp, fp, offs, timeit, res)
    # transpose varm
    cnt = [1024, 1024, 256] if big else [512, 512, 128]
    imap = [1, cnt[0], cnt[0] * cnt[1]]
    n3 = cnt[0] * cnt[1] * cnt[2]
    u3 = torch.empty(n3 * 8, dtype=torch.uint8, device="cuda")
    x3 = torch.empty(n3 * 8, dtype=torch.uint8, device="cuda")
    c3, cp3 = offs(cnt)
    m3, mp3 = offs(imap)
    res.append(("transpose", -1, n3) + timeit(
        lambda: lib.pncx_dev_putn_imap(5, T.NC_DOUBLE, ctypes.c_void_p(x3.data_ptr()), ctypes.c_void_p(u3.data_ptr()),
                                       3, cp3, mp3, T.ITYPE_DOUBLE, fp, ctypes.c_void_p(st.data_ptr()), sp), n3))
    # the same transpose with non-power-of-two extents (strides off the channel interleave)
    for cnt in (([1000, 1000, 268], [1024, 1024, 250], [1000, 1024, 256]) if big else
                ([500, 500, 120], [512, 512, 120], [500, 512, 128])):
        imap = [1, cnt[0], cnt[0] * cnt[1]]
        n5 = cnt[0] * cnt[1] * cnt[2]
        u5 = torch.empty(n5 * 8, dtype=torch.uint8, device="cuda")
        x5 = torch.empty(n5 * 8, dtype=torch.uint8, device="cuda")
        c5, cp5 = offs(cnt)
        m5, mp5 = offs(imap)
        res.append(("transpose_%dx%dx%d" % tuple(cnt), -1, n5) + timeit(
            lambda: lib.pncx_dev_putn_imap(5, T.NC_DOUBLE, ctypes.c_void_p(x5.data_ptr()),
                                           ctypes.c_void_p(u5.data_ptr()), 3, cp5, mp5, T.ITYPE_DOUBLE, fp,
                                           ctypes.c_void_p(st.data_ptr()), sp), n5))
        del u5, x5
    report(res)


def report(res):
    for name, layout, n, ms, gbs in res:
        print(json.dumps({"workload": name, "layout": layout, "n": n, "ms": round(ms, 4),
                          "GB_per_s": round(gbs, 1), "frac_of_8TBs": round(gbs / 8000, 4)}))


def short_runs(args, big, torch, T, pncx, lib, st, sp, fp, offs, timeit, res):
    """short irregular runs (1..7 elements, gaps 0..4) of doubles, 8 copies:
    the default map (4-bit gap steps, k_tgap), the 8- and 16-bit maps, the
    get direction, and the per-element table search without a map"""
    rng = np.random.default_rng(5)
    nb = 1 << (23 if big else 20)
    blen = rng.integers(1, 8, nb)
    disp = np.concatenate([[0], np.cumsum(blen + rng.integers(0, 5, nb))[:-1]]).astype(np.int64) * 8
    span = int(disp[-1]) + int(blen[-1]) * 8
    u4 = torch.empty(span * 8, dtype=torch.uint8, device="cuda")
    dts = pncx.DType(T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(), span)
    n4 = int(blen.sum()) * 8
    x4 = torch.empty(n4 * 8, dtype=torch.uint8, device="cuda")
    c4, cp4 = offs([n4])
    res.append(("short_runs", dts.inq()["layout"], n4) + timeit(
        lambda: lib.pncx_dev_putn_flex(5, T.NC_DOUBLE, ctypes.c_void_p(x4.data_ptr()), ctypes.c_void_p(u4.data_ptr()),
                                       1, cp4, None, 8, dts.handle, fp, ctypes.c_void_p(st.data_ptr()), sp), n4))
    pncx.knob_set("TOFF16", 16)                          # the same typemap with the 16-bit map (round 3)
    dts16 = pncx.DType(T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(), span)
    pncx.knob_set("TOFF16", -1)
    pncx.knob_set("TOFF16", 8)                           # the same typemap with the 8-bit map (round 4)
    dts8 = pncx.DType(T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(), span)
    pncx.knob_set("TOFF16", -1)
    res.append(("short_runs_map8", dts8.inq()["layout"], n4) + timeit(
        lambda: lib.pncx_dev_putn_flex(5, T.NC_DOUBLE, ctypes.c_void_p(x4.data_ptr()), ctypes.c_void_p(u4.data_ptr()),
                                       1, cp4, None, 8, dts8.handle, fp, ctypes.c_void_p(st.data_ptr()), sp), n4))
    res.append(("short_runs_get", dts.inq()["layout"], n4) + timeit(
        lambda: lib.pncx_dev_getn_flex(5, T.NC_DOUBLE, ctypes.c_void_p(x4.data_ptr()), ctypes.c_void_p(u4.data_ptr()),
                                       1, cp4, None, 8, dts.handle, ctypes.c_void_p(st.data_ptr()), sp), n4))
    res.append(("short_runs_map16", dts16.inq()["layout"], n4) + timeit(
        lambda: lib.pncx_dev_putn_flex(5, T.NC_DOUBLE, ctypes.c_void_p(x4.data_ptr()), ctypes.c_void_p(u4.data_ptr()),
                                       1, cp4, None, 8, dts16.handle, fp, ctypes.c_void_p(st.data_ptr()), sp), n4))
    pncx.knob_set("TOFF_MAX_ELEMS", 0)                   # the same typemap without the offset map
    dts2 = pncx.DType(T.ITYPE_DOUBLE, disp.tolist(), blen.tolist(), span)
    pncx.knob_set("TOFF_MAX_ELEMS", -1)
    res.append(("short_runs_search", dts2.inq()["layout"], n4) + timeit(
        lambda: lib.pncx_dev_putn_flex(5, T.NC_DOUBLE, ctypes.c_void_p(x4.data_ptr()), ctypes.c_void_p(u4.data_ptr()),
                                       1, cp4, None, 8, dts2.handle, fp, ctypes.c_void_p(st.data_ptr()), sp), n4))
    del u4, x4


if __name__ == "__main__":
    main()
