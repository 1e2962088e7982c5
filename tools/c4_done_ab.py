"""C4's synchronous call (pncx_dev_batch, swaps only: no statuses to bring
back) waiting on a completion event against the completion kernel and its
host-mapped flag (0, the default), in one process, knob order A B B A per
round; wall time of --steps calls, as bench.py times the call.  Both
settings' outputs are checked (bench.py C4Batch.check).

    python tools/c4_done_ab.py [--rounds 6] [--steps 100]

Round 5 (profiles/r05w_done_ab.txt): an event RECORDED after the batch
kernel (a marker packet) and polled with hipEventQuery was slower (0.2669
against 0.2634 ms per call) and was removed.  Round 6: PNCX_DONE_EVENT=1 is
an event stamped by the batch kernel's own dispatch (hipExtLaunchKernel's
stop event, no extra packet), polled the same way: also slower (0.2625
against 0.2609 ms, profiles/r06h_done_ab.txt), removed with its knob.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--knob", default="DONE_FENCE", help="the 0/1 knob to alternate")
    a = ap.parse_args()
    import torch
    import bench
    from pnetcdf_amd import pncx
    lib = pncx.lib()
    sptr = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    wl = bench.C4Batch(torch, lib, sptr, "sync")
    res = {1: [], 0: []}
    for _ in range(10):
        wl.launch()
    torch.cuda.synchronize()
    for r in range(a.rounds):
        for k in (1, 0, 0, 1):
            pncx.knob_set(a.knob, k)
            for _ in range(5):
                wl.launch()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                wl.launch()
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) * 1e3 / a.steps)
            assert wl.check(), f"DONE_EVENT={k}: wrong output"
    pncx.knob_set(a.knob, -1)
    moved = 256 * (1 << 20) * 6
    for k, v in res.items():
        med = statistics.median(v)
        print(json.dumps({a.knob.lower(): k, "call_ms_median": round(med, 4), "call_ms_min": round(min(v), 4),
                          "frac_of_8TBs": round(moved / (med * 1e-3) / 8e12, 4), "samples": len(v)}), flush=True)


if __name__ == "__main__":
    main()
