"""bench.py -- device-resident XDR swap / NC type-convert throughput on MI355X.

Default workload (BASELINE.json configs[1] / configs[4]): each rank owns one
32 GiB contiguous NC_DOUBLE slab -- at N=1 the config-2 get_vara slab, at N>1
the rank's 32 records (1 GiB each) of the config-5 record variable
v(time=UNLIMITED, 8192, 16384), records 32g..32g+31 on GPU g -- and a step is
one in-place 8-byte big-endian swap pass over it (ncmpii_in_swapn,
convert_swap.m4:160-174), one kernel launch.  Records are independent, so the
slabs shard with no data-path collective (weak scaling); torch.distributed
(RCCL) is used only for the barrier and the max-over-ranks timing.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4]

Prints ONE JSON line on rank 0.  `value` = algorithmic bytes moved (read +
write, 16 B per element) by all ranks / max-over-ranks time, in GiB/s.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEEDS = {"c1": 0x5EED0001, "c2": 0x5EED0002, "c3": 0x5EED0003, "c4": 0x5EED0004, "c5": 0x5EED0005}


def splitmix64_fill(torch, out, seed, chunk=1 << 27):
    """element i = splitmix64(seed + (i+1)*golden), generated on the GPU."""
    n = out.numel()
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        z = torch.arange(s + 1, s + 1 + m, dtype=torch.int64, device=out.device)
        z.mul_(-7046029254386353131).add_(seed)
        z = (z ^ ((z >> 30) & 0x3FFFFFFFF)) * -4658895280553007687
        z = (z ^ ((z >> 27) & 0x1FFFFFFFFF)) * -7723592293110705685
        out[s:s + m] = z ^ ((z >> 31) & 0x1FFFFFFFF)
        del z


def cpu_baseline_swap8(budget_s=12.0, slab_bytes=2 << 30):
    """The oracle's ncmpii_in_swapn restatement (gcc -O2, 1 core) on a
    bounded host sample of the same workload."""
    from oracle import oracle as O
    lib = O.lib()
    buf = np.frombuffer(np.random.default_rng(SEEDS["c2"]).bytes(slab_bytes), dtype=np.uint64).copy()
    n = buf.size
    lib.orc_in_swapn(buf.ctypes.data_as(ctypes.c_void_p), n, 8)  # warm
    passes, t0 = 0, time.perf_counter()
    while True:
        lib.orc_in_swapn(buf.ctypes.data_as(ctypes.c_void_p), n, 8)
        passes += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    moved = 16.0 * n * passes
    return {"value": round(moved / el / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{slab_bytes >> 30} GiB NC_DOUBLE host slab, {passes} in-place 8-byte swap passes "
                      f"in {el:.1f} s (oracle/pncx_oracle.c orc_in_swapn, gcc -O2, 1 thread)"}


def cpu_baseline_swap8_threads(budget_s=4.0, slab_bytes=2 << 30, threads=None):
    """Same restatement on all host cores the box gives one GPU (16): one
    thread per disjoint slice of the slab, the N-ranks-per-node picture of
    BASELINE.md §3.  ctypes releases the GIL during the C call."""
    import threading
    from oracle import oracle as O
    lib = O.lib()
    nt = threads or min(16, os.cpu_count() or 1)
    buf = np.frombuffer(np.random.default_rng(SEEDS["c2"]).bytes(slab_bytes), dtype=np.uint64).copy()
    per = buf.size // nt
    passes = [0] * nt
    t_end = time.perf_counter() + budget_s

    def work(k):
        ptr = ctypes.c_void_p(buf[k * per:].ctypes.data)
        while time.perf_counter() < t_end:
            lib.orc_in_swapn(ptr, per, 8)
            passes[k] += 1
    ths = [threading.Thread(target=work, args=(k,)) for k in range(nt)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    moved = 16.0 * per * sum(passes)
    return {"value": round(moved / el / GIB, 3), "unit": "GiB/s", "cores": nt, "kind": "port",
            "sample": f"{slab_bytes >> 30} GiB slab split over {nt} threads, {sum(passes)} slice passes "
                      f"in {el:.1f} s (orc_in_swapn, gcc -O2)"}


def gather_leg(torch, group, buf, gib, to_cpu=False):
    """Config 5's optional exchange, timed apart from the conversion rate
    (SURVEY §8(e)): every rank's first `gib` GiB of converted records are
    gathered into rank 0 (RCCL gather over xGMI).  Checksums (int64 wrapping
    sums) of what each rank sent are compared on rank 0 with what arrived."""
    n = min(buf.numel(), int(gib * GIB) // 8)
    sl = buf[:n]
    sums = group.all_gather_int(int(sl.sum().item()))
    group.gather_slices(sl, to_cpu)                      # warm the communicator
    torch.cuda.synchronize()
    group.barrier()
    t0 = time.perf_counter()
    got = group.gather_slices(sl, to_cpu)
    torch.cuda.synchronize()
    group.barrier()
    el = group.max([time.perf_counter() - t0])[0]
    ok = True
    if got is not None:
        ok = all(int(g.sum().item()) == s for g, s in zip(got, sums))
        del got
    into = (group.world - 1) * n * 8                      # rank 0's own slice is local
    return {"collective": "gather into rank 0 (RCCL over xGMI)" if not to_cpu else "gather into rank 0 (gloo rehearsal)",
            "bytes_per_rank": n * 8, "bytes_into_rank0": into, "ms": round(el * 1e3, 3),
            "GBps_into_rank0": round(into / el / 1e9, 2), "checksums_ok": ok}


def load_traffic(kernel_key, elems_per_launch):
    """HBM traffic per launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, tools/pmc_summary.py; FETCH_SIZE doubled per
    the gfx950 correction in MI355X_MICROARCH.md §HBM), scaled to this launch
    size.  None when no summary exists."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        e = d["kernels"][kernel_key]
        return e["bytes_per_elem"] * elems_per_launch
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4"])
    ap.add_argument("--slab-gib", type=float, default=32.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--async-batch", action="store_true",
                    help="c4: pncx_dev_batch_async (statuses stay in HBM, calls queue back to back) "
                         "instead of the synchronous pncx_dev_batch")
    ap.add_argument("--gather-gib", type=float, default=1.0,
                    help="N>1, c2: GiB per rank gathered into rank 0 after the timed region (0 = off)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("PNCX_DIST_BACKEND", "nccl") != "nccl":
        local = 0          # rehearsal: every rank on GPU 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("PNCX_DIST_BACKEND", "nccl")   # nccl == RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:   # rehearsal of the N>1 path with several ranks on one GPU
            dist.init_process_group(backend)
    from pnetcdf_amd import nctypes as T
    from pnetcdf_amd import pncx
    from pnetcdf_amd.shard import Group, record_slab
    lib = pncx.lib()
    group = Group(dist, torch.device("cuda", local) if os.environ.get("PNCX_DIST_BACKEND", "nccl") == "nccl"
                  else "cpu")
    stream = torch.cuda.current_stream()
    sptr = ctypes.c_void_p(stream.cuda_stream)

    # ---------------------------------------------------------- workload
    if args.workload == "c2":
        n = int(args.slab_gib * GIB) // 8                      # NC_DOUBLE elements per rank
        rec_elems = 8192 * 16384                               # one 1 GiB record of v(time, 8192, 16384)
        nrec_total = (n // rec_elems) * world
        first_rec, my_recs = record_slab(nrec_total, world, rank)
        buf = torch.empty(n, dtype=torch.int64, device="cuda")
        splitmix64_fill(torch, buf, SEEDS["c5" if world > 1 else "c2"] + first_rec)
        ptr = ctypes.c_void_p(buf.data_ptr())
        bytes_per_elem = 16                                    # 8 R + 8 W
        slab_per_elem = 8                                      # external (file) bytes per element

        def launch():
            rc = lib.pncx_dev_in_swapn(ptr, n, 8, sptr)
            assert rc == 0, rc
        elems = n
        metric_key = "swap8"
        dtype = "u64"
        recs = my_recs
        cfg = {"workload": ("C2: 32 GiB contiguous NC_DOUBLE get_vara, in-place 8-byte swap" if world == 1 else
                            f"C5: NC_DOUBLE record variable v(time={nrec_total}, 8192, 16384), "
                            f"{recs} x 1 GiB records per GPU, in-place 8-byte swap"),
               "slab_gib_per_gpu": args.slab_gib, "elements_per_gpu": n, "xtype": "NC_DOUBLE",
               "itype": "double", "records_per_gpu": recs,
               "parallelism": f"records sharded one slab per GPU x{world}, no data-path collective"}
    elif args.workload == "c3":
        n = 1 << 31                                            # NC_INT elements
        xb = torch.empty(n // 2, dtype=torch.int64, device="cuda")
        splitmix64_fill(torch, xb, SEEDS["c3"] + rank)
        ib = torch.empty(n, dtype=torch.float64, device="cuda")
        st = torch.zeros(1, dtype=torch.int32, device="cuda")
        px, pi, ps = (ctypes.c_void_p(t.data_ptr()) for t in (xb, ib, st))

        def launch():
            rc = lib.pncx_dev_getn(5, T.NC_INT, px, pi, n, T.ITYPE_DOUBLE, ps, sptr)
            assert rc == 0, rc
        elems = n
        bytes_per_elem = 12
        slab_per_elem = 4
        metric_key = "get_int_double"
        dtype = "int32->f64"
        cfg = {"workload": "C3: NC_INT on disk read via get_vara_double, fused 4-byte swap + int32->double",
               "elements_per_gpu": n, "xtype": "NC_INT", "itype": "double", "parallelism": f"x{world}"}
    else:
        nvar, nel = 256, 1 << 20
        segs = []
        keep = []
        for v in range(nvar):
            if v % 2 == 0:
                xt, it, isz = T.NC_SHORT, T.ITYPE_SHORT, 2
            else:
                xt, it, isz = T.NC_FLOAT, T.ITYPE_FLOAT, 4
            ib = torch.randint(-2**31, 2**31 - 1, (nel * isz // 4,), dtype=torch.int32, device="cuda")
            xb = torch.empty(nel * isz, dtype=torch.uint8, device="cuda")
            keep += [ib, xb]
            segs.append(pncx.Seg(T.PNCX_PUT, 5, xt, it, nel, xb.data_ptr(), ib.data_ptr(), None))
        arr = (pncx.Seg * nvar)(*segs)
        stv = (ctypes.c_int * nvar)()
        dstv = torch.zeros(nvar, dtype=torch.int32, device="cuda")
        dstp = ctypes.c_void_p(dstv.data_ptr())

        def launch():
            if args.async_batch:
                rc = lib.pncx_dev_batch_async(arr, nvar, dstp, sptr)
            else:
                rc = lib.pncx_dev_batch(arr, nvar, stv, sptr)
            assert rc == 0, rc
        elems = nvar * nel
        bytes_per_elem = 6                                     # avg of 2*2 (short) and 2*4 (float)
        slab_per_elem = 3
        metric_key = "batch_c4"
        dtype = "i16/f32"
        cfg = {"workload": "C4: iput_vara batch, 256 variables x 2^20 elements, NC_SHORT/NC_FLOAT mixed",
               "variables": nvar, "elements_per_var": nel, "parallelism": f"x{world}",
               "call": "pncx_dev_batch_async (statuses in HBM)" if args.async_batch
               else "pncx_dev_batch (statuses to host, synchronous)"}

    torch.cuda.synchronize()
    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize()
    if args.workload == "c4" and not args.async_batch:
        # the batch call also copies the statuses back and waits: its kernel
        # time comes from HIP events the library records around the launch
        lib.pncx_dev_batch_timing(1)

    # ---------------------------------------------------------- timed region
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    group.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        evs[k][0].record(stream)
        launch()
        evs[k][1].record(stream)
    torch.cuda.synchronize()
    group.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    call_ms = None
    if args.workload == "c4" and args.async_batch:
        assert int(dstv.abs().sum().item()) == 0        # swaps: no segment may report NC_ERANGE
    if args.workload == "c4" and not args.async_batch:
        tot, calls = ctypes.c_double(), ctypes.c_longlong()
        assert lib.pncx_dev_batch_kernel_ms(ctypes.byref(tot), ctypes.byref(calls)) == 0 and calls.value == args.steps
        call_ms, kern_ms = kern_ms, tot.value / calls.value
        lib.pncx_dev_batch_timing(0)
    elapsed, kern_ms = group.max([elapsed, kern_ms])         # max over ranks

    gather = None
    if world > 1 and args.gather_gib > 0 and args.workload == "c2":
        gather = gather_leg(torch, group, buf, args.gather_gib,
                            to_cpu=os.environ.get("PNCX_DIST_BACKEND", "nccl") != "nccl")

    moved = float(bytes_per_elem) * elems * world * args.steps
    value = moved / elapsed / GIB
    ms_per_step = elapsed * 1e3 / args.steps
    achieved = bytes_per_elem * elems / (kern_ms * 1e-3) / 1e9           # GB/s per GPU, per launch
    traffic = load_traffic(metric_key, elems)

    if rank == 0:
        cpu = cpu_all = None
        if world == 1 and not args.no_cpu_baseline and args.workload == "c2":
            cpu = cpu_baseline_swap8(args.cpu_budget)
            cpu_all = cpu_baseline_swap8_threads()
        line = {
            "metric": "GiB/s device-resident swap+type-convert, 2/4/8-byte NC arrays",
            "value": round(value, 2),
            "slab_GiBps": round(value * slab_per_elem / bytes_per_elem, 2),   # external bytes / t
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (splitmix64 bit patterns generated on the GPU)",
            "config": cfg,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel_ms_avg": round(kern_ms, 4),
                         **({"call_ms_avg": round(call_ms, 4)} if call_ms is not None else {}),
                         "algorithmic_bytes_per_launch": bytes_per_elem * elems},
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
        }
        if gather is not None:
            line["gather"] = gather
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
