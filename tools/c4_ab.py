"""A/B of two builds of libpncx.so on the C4 batch, in one process,
interleaved round by round (process-to-process spread on this pool exceeds
the effects being measured, so separate bench runs cannot decide them).

A is the in-tree library; B is another build of the same sources, e.g.

    make -C pnetcdf_amd/csrc OUT=$PWD/tools/ab OBJ=$PWD/tools/ab/obj \\
        "HIPFLAGS=--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -DPNCX_BATCH_REMAP=0" \\
        $PWD/tools/ab/libpncx.so
    python tools/c4_ab.py --b tools/ab/libpncx.so [--b other.so] [--rounds 6] [--steps 20]

Each library gets its own C4 buffers (bench.py's C4Batch: torch allocations,
splitmix64 data) for the synchronous, asynchronous and NC_ERANGE workloads;
each sample is bench.py's measure() (kernel time from the library's
dispatch-stamped events, call time from the wall clock).
"""
import argparse
import copy
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", required=True, action="append",
                    help="another build of libpncx.so (repeatable: B, C, ...)")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--modes", default="sync,async,erange")
    a = ap.parse_args()
    import torch
    import bench
    from pnetcdf_amd import pncx
    from pnetcdf_amd.shard import Group
    # RTLD_DEEPBIND: each other build must call its own kernel launchers --
    # without it the first library (loaded RTLD_GLOBAL) interposes every
    # pncxk_* symbol the others call, so their host code runs A's kernels
    libs = {"A": pncx.lib()}
    for k, path in enumerate(a.b):
        libs[chr(ord("B") + k)] = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL | os.RTLD_DEEPBIND)
    stream = torch.cuda.current_stream()
    sptr = ctypes.c_void_p(stream.cuda_stream)
    group = Group()
    modes = tuple(a.modes.split(","))
    # one buffer set per library and mode; in round r library k runs on the
    # buffer set of library (k + r) mod n, so each build meets every placement
    # (placement alone moved the same kernels by 3 % between buffer sets)
    names = list(libs)
    sets = {(i, m): bench.C4Batch(torch, libs["A"], sptr, m) for i in range(len(names)) for m in modes}

    def view(w, L):
        v = copy.copy(w)
        nvar, arr = w._nvar, w._arr
        if w._async:
            dp = ctypes.c_void_p(w._tdst.data_ptr())
            v.launch = lambda: bench._ok(L.pncx_dev_batch_async(arr, nvar, dp, sptr))
        else:
            stv = w._stv
            v.launch = lambda: bench._ok(L.pncx_dev_batch(arr, nvar, stv, sptr),
                                         w._T.NC_ERANGE if w._erange else 0)
        return v

    wls = {}
    res = {}
    for r in range(a.rounds):
        for m in modes:
            for ki, (k, L) in enumerate(libs.items()):
                wls[(k, m)] = view(sets[((ki + r) % len(names), m)], L)
                try:
                    el, km, cm = bench.measure(torch, L, group, stream, wls[(k, m)], a.steps, 3)
                except AssertionError as e:
                    raise SystemExit(f"library {k} ({m}): {e!r}")
                assert wls[(k, m)].check(), (k, m)
                res.setdefault((m, k), []).append((km, el * 1e3 / a.steps))
    for (m, k), v0 in sorted(res.items()):
        v = v0[1:]                     # round 0: the first K calls after the buffers were made
        w = wls[(k, m)]
        algo = w.bytes_per_elem * w.elems
        km = statistics.median(x[0] for x in v)
        cm = statistics.median(x[1] for x in v)
        print(json.dumps({"mode": m, "lib": k, "kernel_ms_median": round(km, 4), "call_ms_median": round(cm, 4),
                          "kernel_frac": round(algo / (km * 1e-3) / 8e12, 4),
                          "call_frac": round(algo / (cm * 1e-3) / 8e12, 4),
                          "kernel_ms_all": [round(x[0], 4) for x in v0],
                          "call_ms_all": [round(x[1], 4) for x in v0]}), flush=True)


if __name__ == "__main__":
    main()
