"""Where does C4's gap to C2 come from: size (launch ramp and drain) or
out-of-place traffic (reads and writes in different DRAM rows)?

The product's 4-byte swap kernel (pncx_dev_in_swapn / pncx_dev_swapn, one
k_tile<SwapOp<4>> launch) over S bytes per side, in place (src == dst) and out
of place, for several S, interleaved round by round in one process.  Each
measurement is `reps` launches back to back between two events on the launch
stream (steady state), reported as algorithmic bytes (2 S per launch) / time.

    python tools/oop_probe.py [--rounds 4] [--reps 10] [--sizes-mib 768,3072,12288]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sizes-mib", default="768,3072,12288")
    a = ap.parse_args()
    import torch
    from pnetcdf_amd import pncx
    sizes = [int(s) << 20 for s in a.sizes_mib.split(",")]
    big = max(sizes)
    src = torch.randint(-2**31, 2**31 - 1, (big // 4,), dtype=torch.int32, device="cuda")
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream()
    res = {}
    for r in range(a.rounds):
        for S in sizes:
            n = S // 4
            for mode in ("inplace", "oop"):
                if mode == "inplace":
                    f = lambda: pncx.dev_in_swapn(src, n, 4, stream=stream)
                else:
                    f = lambda: pncx.dev_swapn(dst, src, n, 4, stream=stream)
                f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.reps):
                    f()
                e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res.setdefault((S, mode), []).append(2 * S / (ms * 1e-3) / 1e9)
    for (S, mode), v in sorted(res.items()):
        print(json.dumps({"bytes_per_side": S, "mode": mode, "GBps_median": round(statistics.median(v), 1),
                          "GBps_all": [round(x, 1) for x in v],
                          "frac_median": round(statistics.median(v) / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
