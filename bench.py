"""bench.py -- device-resident XDR swap / NC type-convert throughput on MI355X.

Headline workload (BASELINE.json configs[1] / configs[4]): each rank owns one
32 GiB contiguous NC_DOUBLE slab -- at N=1 the config-2 get_vara slab, at N>1
the rank's 32 records (1 GiB each) of the config-5 record variable
v(time=UNLIMITED, 8192, 16384), records 32g..32g+31 on GPU g -- and a step is
one in-place 8-byte big-endian swap pass over it (ncmpii_in_swapn,
convert_swap.m4:160-174), one kernel launch.  Records are independent, so the
slabs shard with no data-path collective (weak scaling); torch.distributed
(RCCL) is used only for the barrier and the max-over-ranks timing.

At N=1 the same run then measures the other single-GPU configs, one after
another with each workload's buffers freed before the next (`workloads` in
the JSON line; none of them feeds `value`):
    c3        2^31 NC_INT read as double (fused 4-byte swap + int32->double)
    c4        256 x 2^20 iput batch, NC_SHORT/NC_FLOAT same-type (pncx_dev_batch)
    c4_async  the same through pncx_dev_batch_async (statuses stay in HBM)
    c4_erange SURVEY §8(d)'s secondary variant: the NC_SHORT variables come
              from float values uniform in [-40000, 40000] (~18% NC_ERANGE + fill)

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c4|c4_async|c4_erange]

--gpus N without a torch.distributed launcher (no WORLD_SIZE in the
environment) starts N ranks itself: torch.distributed.run as a child
process, before this process touches the GPU, and exits with its status.

Prints ONE JSON line on rank 0.  `value` = algorithmic bytes moved (read +
write, 16 B per element) by all ranks / max-over-ranks time, in GiB/s.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEEDS = {"c1": 0x5EED0001, "c2": 0x5EED0002, "c3": 0x5EED0003, "c4": 0x5EED0004, "c5": 0x5EED0005}
EXTRA = ("c3", "c4", "c4_async", "c4_erange")


# --------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_cmd(argv, nproc, port):
    """torch.distributed.run command that starts `nproc` ranks of this script
    with the same arguments (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(nproc, argv):
    """Start the N ranks as a child process group and return its exit code.
    This process has not initialised the GPU (nothing here imports torch.cuda
    state), and it waits rather than exec'ing."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(launch_cmd(argv, nproc, _free_port()), env=env)


# --------------------------------------------------------------- helpers
def splitmix64_fill(torch, out, seed, chunk=1 << 27, base=0):
    """element i = splitmix64(seed + (base+i+1)*golden), generated on the GPU."""
    n = out.numel()
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        z = torch.arange(base + s + 1, base + s + 1 + m, dtype=torch.int64, device=out.device)
        z.mul_(-7046029254386353131).add_(seed)
        z = (z ^ ((z >> 30) & 0x3FFFFFFFF)) * -4658895280553007687
        z = (z ^ ((z >> 27) & 0x1FFFFFFFFF)) * -7723592293110705685
        out[s:s + m] = z ^ ((z >> 31) & 0x1FFFFFFFF)
        del z


def splitmix_uniform(torch, out, seed, lo, hi):
    """float32 values uniform in [lo, hi) from splitmix64 bits (the top 24)."""
    bits = torch.empty(out.numel(), dtype=torch.int64, device=out.device)
    splitmix64_fill(torch, bits, seed)
    u = ((bits >> 40) & 0xFFFFFF).to(torch.float64) * (1.0 / (1 << 24))
    out.copy_((lo + (hi - lo) * u).to(torch.float32))
    del bits, u


def host_cpu():
    """The host CPU model and the logical CPUs visible (report
    nproc and the model beside the CPU baselines)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "nproc": os.cpu_count()}


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
                      f"in {el:.1f} s (oracle/pncx_oracle.c orc_in_swapn, gcc -O2, 1 thread)",
            "host": host_cpu()}


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


def cpu_run(jobs, threads, budget_s):
    """Time a list of (ctypes call, algorithmic bytes) jobs on `threads` host
    threads: thread k runs jobs k, k+T, ... over and over until the budget
    is spent (ctypes releases the GIL inside each call).  Returns
    (GiB/s moved, jobs completed, seconds)."""
    import threading
    done = [0] * threads
    moved = [0.0] * threads
    t_end = time.perf_counter() + budget_s

    def work(k):
        mine = jobs[k::threads]
        while mine and time.perf_counter() < t_end:
            for call, nbytes in mine:
                call()
                done[k] += 1
                moved[k] += nbytes
    for call, _ in jobs[:threads]:     # warm: first touch of the host pages
        call()
    ths = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    return sum(moved) / el / GIB, sum(done), el


def cpu_baseline_jobs(name, jobs, threads, budget_s, sample):
    v, calls, el = cpu_run(jobs, threads, budget_s)
    return {"value": round(v, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{sample}; {calls} oracle calls in {el:.1f} s on {threads} thread(s) "
                      f"(oracle/pncx_oracle.c, gcc -O2)"}


def cpu_c3_jobs(lib, n=1 << 26, pieces=16, seed=0):
    """NC_INT -> double getn (ncmpii_getn_NC_INT, ncx.m4:2429-2495) on a
    2^26-element host sample cut into `pieces` disjoint slices."""
    from pnetcdf_amd import nctypes as T
    xb = np.frombuffer(np.random.default_rng(seed).bytes(n * 4), np.uint8).copy()
    ib = np.empty(n * 8, np.uint8)
    per = n // pieces
    jobs = []
    for k in range(pieces):
        xp, ip = xb.ctypes.data + k * per * 4, ib.ctypes.data + k * per * 8
        jobs.append((lambda xp=xp, ip=ip: lib.orc_getn(5, T.NC_INT, xp, ip, per, T.ITYPE_DOUBLE), 12.0 * per))
    return jobs, (xb, ib)


def cpu_c4_jobs(lib, erange, nel=1 << 20, nvar=256, seed=0):
    """The C4 batch on the host: one ncmpii_putn_NC_<X> per iput request
    (ncmpio_i_getput.m4:238-239 -> convert_swap.m4:202-330): 128 NC_SHORT
    (from short, or from float in [-40000, 40000] for the secondary
    variant, with the NC_SHORT fill) and 128 NC_FLOAT same-type requests of
    2^20 elements, the whole workload in host memory."""
    from pnetcdf_amd import nctypes as T
    rng = np.random.default_rng(seed)
    keep, jobs = [], []
    fill = np.frombuffer(T.fill_bytes(T.NC_SHORT) + b"\0" * 8, np.uint8).copy()
    keep.append(fill)
    for v in range(nvar):
        if v % 2 == 0 and erange:
            ib = rng.uniform(-40000.0, 40000.0, nel).astype(np.float32)
            xt, it, isz, xsz = T.NC_SHORT, T.ITYPE_FLOAT, 4, 2
        elif v % 2 == 0:
            ib = np.frombuffer(rng.bytes(nel * 2), np.int16).copy()
            xt, it, isz, xsz = T.NC_SHORT, T.ITYPE_SHORT, 2, 2
        else:
            ib = np.frombuffer(rng.bytes(nel * 4), np.float32).copy()
            xt, it, isz, xsz = T.NC_FLOAT, T.ITYPE_FLOAT, 4, 4
        xb = np.empty(nel * xsz, np.uint8)
        keep += [ib, xb]
        jobs.append((lambda xt=xt, it=it, xp=xb.ctypes.data, ip=ib.ctypes.data:
                     lib.orc_putn(5, xt, xp, ip, nel, it, fill.ctypes.data), float((isz + xsz) * nel)))
    return jobs, keep


PCIE_GBPS = 57.5     # pinned H2D on the MI355X host, profiles/r01_pcie.json


def gather_leg(torch, group, buf, gib, chunk_gib, to_cpu=False):
    """Config 5's exchange, timed apart from the conversion rate (SURVEY
    §8(e)): every rank's first `gib` GiB of converted records are gathered
    into rank 0 (RCCL gather over xGMI), streamed in chunks of `chunk_gib`
    GiB per rank through one reused receive buffer, so the whole slab (the
    config's 224 GiB into rank 0 at N=8) moves without rank 0 holding it.
    Checksums (int64 wrapping sums) of every chunk each rank sent are
    compared on rank 0 with what arrived."""
    n = min(buf.numel(), int(gib * GIB) // 8)
    step = max(1, min(n, int(chunk_gib * GIB) // 8))
    chunks = [(s, min(step, n - s)) for s in range(0, n, step)]
    sums = [group.all_gather_int(int(buf[s:s + m].sum().item())) for s, m in chunks]
    group.gather_slices(buf[:min(step, n)], to_cpu)          # warm the communicator
    torch.cuda.synchronize()
    group.barrier()
    arrived = []
    t0 = time.perf_counter()
    for k, (s, m) in enumerate(chunks):
        got = group.gather_slices(buf[s:s + m], to_cpu)
        if got is not None:              # rank 0: checksum kernels queue behind the gather (~2% of its time)
            arrived.append([g.sum() for g in got])
        del got
    torch.cuda.synchronize()
    group.barrier()
    el = group.max([time.perf_counter() - t0])[0]
    ok = all(int(a.item()) == want for got_k, sums_k in zip(arrived, sums) for a, want in zip(got_k, sums_k))
    into = (group.world - 1) * n * 8                         # rank 0's own slice is local
    rate = into / el / 1e9
    return {"collective": "gather into rank 0 (RCCL over xGMI)" if not to_cpu else "gather into rank 0 (gloo rehearsal)",
            "bytes_per_rank": n * 8, "bytes_into_rank0": into, "chunk_bytes_per_rank": step * 8,
            "chunks": len(chunks), "ms": round(el * 1e3, 3), "GBps_into_rank0": round(rate, 2),
            "checksums_ok": ok,
            # xGMI into one GPU is ~7 x 153 GB/s; a gather that does
            # not beat the PCIe link (57.5 GB/s H2D, profiles/r01_pcie.json)
            # went through the host, not xGMI
            "via_xgmi": (not to_cpu) and rate > PCIE_GBPS, "pcie_ceiling_GBps": PCIE_GBPS,
            "note": "timed region includes one int64 sum kernel per arrived chunk on rank 0"}


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


def traffic_source():
    """Which PMC pass roofline.traffic comes from: the summary file and the
    round tag tools/pmc_summary.py wrote into it."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        return {"file": "profiles/pmc_traffic.json", "round": d.get("round"), "pmc_csv": d.get("source")}
    except Exception:
        return None


# --------------------------------------------------------------- workloads
class Workload:
    """One single-GPU configuration: buffers in HBM, a launch() = one step,
    the algorithmic bytes of a step, and a check() of the last step."""
    lib_timed = False          # kernel time from the library's own events (pncx_dev_batch)

    def check(self):
        return True

    def free(self):
        for k in list(vars(self)):
            if k.startswith("_t"):
                setattr(self, k, None)


class C2Swap(Workload):
    def __init__(self, torch, lib, sptr, slab_gib, world, rank):
        from pnetcdf_amd.shard import record_slab
        self.check_desc = ""
        n = int(slab_gib * GIB) // 8                           # NC_DOUBLE elements per rank
        rec_elems = 8192 * 16384                               # one 1 GiB record of v(time, 8192, 16384)
        nrec_total = (n // rec_elems) * world
        first_rec, my_recs = record_slab(nrec_total, world, rank)
        self._tbuf = torch.empty(n, dtype=torch.int64, device="cuda")
        self._seed = SEEDS["c5" if world > 1 else "c2"] + first_rec
        splitmix64_fill(torch, self._tbuf, self._seed)
        ptr = ctypes.c_void_p(self._tbuf.data_ptr())
        self.passes = 0

        def launch():
            _ok(lib.pncx_dev_in_swapn(ptr, n, 8, sptr))
            self.passes += 1
        self.launch = launch
        self._torch, self._n = torch, n
        self.elems, self.bytes_per_elem, self.slab_per_elem = n, 16, 8
        self.metric_key, self.dtype = "swap8", "u64"
        self.check_desc = ("every element of the slab against the splitmix64 values regenerated on the GPU, "
                           "byte-reversed by torch when the pass count is odd")
        self.kernel = "k_tile<SwapOp<8>, true>"
        self.cfg = {"workload": ("C2: 32 GiB contiguous NC_DOUBLE get_vara, in-place 8-byte swap" if world == 1 else
                                 f"C5: NC_DOUBLE record variable v(time={nrec_total}, 8192, 16384), "
                                 f"{my_recs} x 1 GiB records per GPU, in-place 8-byte swap"),
                    "slab_gib_per_gpu": slab_gib, "elements_per_gpu": n, "xtype": "NC_DOUBLE",
                    "itype": "double", "records_per_gpu": my_recs,
                    "parallelism": f"records sharded one slab per GPU x{world}, no data-path collective"}


    def check(self):
        """Every element: the in-place swap is an involution, so after an
        odd number of passes element i is the byte reversal of the
        splitmix64 value the slab was filled with, after an even number the
        value itself.  The expected slab is regenerated on the GPU in 1 GiB
        chunks and byte-reversed by torch (flip of the 8 bytes), independent
        of the kernel under test."""
        torch = self._torch
        odd = self.passes % 2 == 1
        chunk = 1 << 27
        for s in range(0, self._n, chunk):
            m = min(chunk, self._n - s)
            exp = torch.empty(m, dtype=torch.int64, device="cuda")
            splitmix64_fill(torch, exp, self._seed, base=s)
            if odd:
                exp = exp.view(torch.uint8).view(m, 8).flip(1).contiguous().view(torch.int64).view(m)
            if not torch.equal(exp, self._tbuf[s:s + m]):
                return False
            del exp
        return True


class C3IntDouble(Workload):
    def __init__(self, torch, lib, sptr, rank=0):
        from pnetcdf_amd import nctypes as T
        n = 1 << 31                                            # NC_INT elements
        self._txb = torch.empty(n // 2, dtype=torch.int64, device="cuda")
        splitmix64_fill(torch, self._txb, SEEDS["c3"] + rank)
        self._tib = torch.empty(n, dtype=torch.float64, device="cuda")
        self._tst = torch.zeros(1, dtype=torch.int32, device="cuda")
        px, pi, ps = (ctypes.c_void_p(t.data_ptr()) for t in (self._txb, self._tib, self._tst))
        self.launch = lambda: _ok(lib.pncx_dev_getn(5, T.NC_INT, px, pi, n, T.ITYPE_DOUBLE, ps, sptr))
        self.elems, self.bytes_per_elem, self.slab_per_elem = n, 12, 4
        self.metric_key, self.dtype = "get_int_double", "int32->f64"
        self.check_desc = "every element against torch's byte flip + int32->double cast of the input; status NC_NOERR"
        self.kernel = "k_tile<GetOp<NC_INT, double>, true>"
        self.cfg = {"workload": "C3: NC_INT on disk read via get_vara_double, fused 4-byte swap + int32->double",
                    "elements_per_gpu": n, "xtype": "NC_INT", "itype": "double"}
        self._n = n
        self._torch = torch

    def check(self):
        """int->double is exact and never ERANGE: every element equals the
        byte-reversed int32 of the input (torch byte flip + cast, 2^27
        elements at a time), and the status word stays NC_NOERR"""
        torch = self._torch
        xi = self._txb.view(torch.int32)
        chunk = 1 << 27
        for s in range(0, self._n, chunk):
            m = min(chunk, self._n - s)
            b = xi[s:s + m].view(torch.uint8).view(m, 4).flip(1).contiguous().view(torch.int32).view(m)
            if not torch.equal(b.to(torch.float64), self._tib[s:s + m]):
                return False
            del b
        return int(self._tst.item()) == 0


class C4Batch(Workload):
    """256 iput_vara requests of 2^20 elements, flushed by one wait_all: one
    batched conversion (pncx_dev_batch / pncx_dev_batch_async).  erange:
    the NC_SHORT variables take float input in [-40000, 40000]."""

    def __init__(self, torch, lib, sptr, mode="sync", rank=0):
        from pnetcdf_amd import nctypes as T
        from pnetcdf_amd import pncx
        nvar, nel = 256, 1 << 20
        segs, self._tkeep, self._fills = [], [], []
        self._erange = mode == "erange"
        for v in range(nvar):
            if v % 2 == 0 and self._erange:
                xt, it, isz = T.NC_SHORT, T.ITYPE_FLOAT, 4
                ib = torch.empty(nel, dtype=torch.float32, device="cuda")
                splitmix_uniform(torch, ib, SEEDS["c4"] + 1000 * rank + v, -40000.0, 40000.0)
            else:
                xt, it, isz = (T.NC_SHORT, T.ITYPE_SHORT, 2) if v % 2 == 0 else (T.NC_FLOAT, T.ITYPE_FLOAT, 4)
                ib = torch.empty(nel * isz // 8, dtype=torch.int64, device="cuda")
                splitmix64_fill(torch, ib, SEEDS["c4"] + 1000 * rank + v)
            xb = torch.empty(nel * T.xlen(xt), dtype=torch.uint8, device="cuda")
            self._tkeep += [ib, xb]
            fill = np.frombuffer(T.fill_bytes(xt) + b"\0" * 8, np.uint8).copy()   # native order, 8-byte slot
            self._fills.append(fill)
            segs.append(pncx.Seg(T.PNCX_PUT, 5, xt, it, nel, xb.data_ptr(), ib.data_ptr(), fill.ctypes.data))
        self._arr = (pncx.Seg * nvar)(*segs)
        self._stv = (ctypes.c_int * nvar)()
        self._tdst = torch.zeros(nvar, dtype=torch.int32, device="cuda")
        dstp = ctypes.c_void_p(self._tdst.data_ptr())
        self._async = mode == "async"
        self._T, self._nvar, self._torch, self._lib = T, nvar, torch, lib
        arr, stv = self._arr, self._stv
        if self._async:
            self.launch = lambda: _ok(lib.pncx_dev_batch_async(arr, nvar, dstp, sptr))
        else:
            self.launch = lambda: _ok(lib.pncx_dev_batch(arr, nvar, stv, sptr), T.NC_ERANGE if self._erange else 0)
        self.lib_timed = True        # kernel time: the library's dispatch-stamped events
        # algorithmic bytes: isz + xsz per element, summed over the variables
        per_pair = (4 + 2) + (4 + 4) if self._erange else (2 + 2) + (4 + 4)
        self.elems = nvar * nel
        self.bytes_per_elem = per_pair / 2.0
        self.slab_per_elem = 3
        self.metric_key = "batch_c4_erange" if self._erange else "batch_c4"
        self.check_desc = ("all 256 statuses and every output element against torch's byte flip (same-type) or "
                           "trunc + NC_SHORT fill outside [-32768, 32767] (float -> NC_SHORT)")
        self.dtype = "f32->i16/f32" if self._erange else "i16/f32"
        self.kernel = ("k_batch<PutOp<NC_SHORT, float>> + k_batch_swapmix" if self._erange
                       else "k_batch_swapmix")
        self.cfg = {"workload": ("C4 secondary: iput_vara batch, 128 NC_SHORT vars from float in [-40000, 40000] "
                                 "(~18% NC_ERANGE + fill) + 128 NC_FLOAT vars, 2^20 elements each" if self._erange
                                 else "C4: iput_vara batch, 256 variables x 2^20 elements, NC_SHORT/NC_FLOAT mixed"),
                    "variables": nvar, "elements_per_var": nel,
                    "call": "pncx_dev_batch_async (statuses in HBM)" if self._async
                    else "pncx_dev_batch (statuses to host, synchronous)"}

    def check(self):
        """Statuses (NC_ERANGE exactly on the float -> NC_SHORT variables of
        the secondary variant) and every output element: a same-type
        variable is its input with each element's bytes reversed; a float
        -> NC_SHORT variable is trunc(x) big-endian, or the NC_SHORT fill
        -32767 where x is outside [-32768, 32767] (NCX_PUT1F, ncx.m4:604-625;
        computed here by torch, independent of the kernels)"""
        T, torch = self._T, self._torch
        exp = [T.NC_ERANGE if (self._erange and v % 2 == 0) else 0 for v in range(self._nvar)]
        got = self._tdst.cpu().tolist() if self._async else list(self._stv)
        if got != exp:
            return False
        for v in range(self._nvar):
            ib, xb = self._tkeep[2 * v], self._tkeep[2 * v + 1]
            if v % 2 == 0 and self._erange:
                f = ib
                o = (f > 32767.0) | (f < -32768.0)
                want = torch.where(o, torch.full_like(f, -32767.0), f).to(torch.int32).to(torch.int16)
                esz = 2
            else:
                esz = 2 if v % 2 == 0 else 4
                want = ib
            w = want.contiguous().view(torch.uint8).view(-1, esz).flip(1).contiguous().view(-1)
            if not torch.equal(w, xb):
                return False
        return True


def _ok(rc, allowed=0):
    assert rc == 0 or rc == allowed, rc


def make_workload(name, torch, lib, sptr, args, world, rank):
    if name == "c2":
        return C2Swap(torch, lib, sptr, args.slab_gib, world, rank)
    if name == "c3":
        return C3IntDouble(torch, lib, sptr, rank)
    if name == "c4":
        return C4Batch(torch, lib, sptr, "async" if args.async_batch else "sync", rank)
    if name == "c4_async":
        return C4Batch(torch, lib, sptr, "async", rank)
    if name == "c4_erange":
        return C4Batch(torch, lib, sptr, "erange", rank)
    raise ValueError(name)


def measure(torch, lib, group, stream, wl, steps, warmup):
    """W untimed warmups, then K steps between barrier + synchronize; HIP
    events on the kernel's stream around every launch (for the synchronous
    batch call the library's own kernel events, in a second pass).  Returns
    (max-over-ranks wall seconds, kernel ms per launch, call ms or None)."""
    torch.cuda.synchronize()
    for _ in range(warmup):
        wl.launch()
    torch.cuda.synchronize()
    # The synchronous batch call returns after its kernels, so the wall clock
    # times the calls; the library's kernel events (stamped by the kernels'
    # own dispatches) add ~9 us to each synchronous call, so they run in a
    # second pass of the same K calls (tools/c4_call_probe.py).
    evs = [] if wl.lib_timed else \
        [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    group.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if wl.lib_timed:
        for k in range(steps):
            wl.launch()
    else:
        for k in range(steps):
            evs[k][0].record(stream)
            wl.launch()
            evs[k][1].record(stream)
    torch.cuda.synchronize()
    group.barrier()
    elapsed = time.perf_counter() - t0
    call_ms = None
    if wl.lib_timed:
        lib.pncx_dev_batch_timing(1)
        for k in range(steps):
            wl.launch()
        tot, calls = ctypes.c_double(), ctypes.c_longlong()
        assert lib.pncx_dev_batch_kernel_ms(ctypes.byref(tot), ctypes.byref(calls)) == 0 and calls.value == steps
        call_ms, kern_ms = elapsed * 1e3 / steps, tot.value / calls.value
        lib.pncx_dev_batch_timing(0)
    else:
        kern_ms = sum(a.elapsed_time(b) for a, b in evs) / steps
    wl.rank_kernel_ms = kern_ms
    elapsed, kern_ms = group.max([elapsed, kern_ms])
    return elapsed, kern_ms, call_ms


def summary(wl, elapsed, kern_ms, call_ms, steps, world):
    moved = float(wl.bytes_per_elem) * wl.elems * world * steps
    value = moved / elapsed / GIB
    achieved = wl.bytes_per_elem * wl.elems / (kern_ms * 1e-3) / 1e9         # GB/s per GPU, per launch
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": load_traffic(wl.metric_key, wl.elems),
            "traffic_source": traffic_source(),
            "kernel": wl.kernel, "kernel_ms_avg": round(kern_ms, 4),
            "algorithmic_bytes_per_launch": int(wl.bytes_per_elem * wl.elems)}
    if call_ms is not None:
        roof["call_ms_avg"] = round(call_ms, 4)
    return value, elapsed * 1e3 / steps, roof


def c1_leg(reps=21, n=1 << 20):
    """BASELINE configs[0]: 1-D 2^20 NC_INT ncmpi_put_vara_int_all +
    ncmpi_get_vara_int_all through libpnetcdf.so (tests/mpi/api_check
    c1bench, one MPI rank, a file on tmpfs /dev/shm), with host buffers
    (8 I/O threads, and 1 to match the reference's single writer) and with
    hipMalloc'ed buffers.  Rates are external (file) bytes / call time."""
    exe = os.path.join(ROOT, "tests", "mpi", "api_check")
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    path = os.path.join(shm, f"pncx_c1_{os.getpid()}.nc")
    res = {}
    xbytes = 4.0 * n
    for key, dev, threads in (("host_8_io_threads", 0, None), ("host_1_io_thread", 0, "1"), ("device_buffers", 1, None)):
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if threads is not None:
            env["PNCX_IO_THREADS"] = threads
        r = subprocess.run([exe, "c1bench", path, str(n), str(reps), str(dev)], capture_output=True, text=True,
                           timeout=300, env=env)
        if r.returncode != 0:
            res[key] = {"error": r.returncode, "stderr": r.stderr[-400:]}
            continue
        o = json.loads(r.stdout.strip().splitlines()[-1])
        res[key] = {"put_ms": o["put_ms_median"], "get_ms": o["get_ms_median"],
                    "put_GiBps": round(xbytes / (o["put_ms_median"] * 1e-3) / GIB, 3),
                    "get_GiBps": round(xbytes / (o["get_ms_median"] * 1e-3) / GIB, 3), "errors": o["errors"]}
        res["var_offset"] = o["var_offset"]
    return res, path


def c1_reference_sequence(path, var_offset, reps=21, n=1 << 20):
    """The reference's C1 sequence restated on one host thread and timed in
    C (oracle/ref_sequence.c, the cpu_baseline of the c1 leg; an oracle
    restatement of the reference loop, not the reference binary): put = swap
    the user buffer in place, pwrite, swap it back (ncmpio_getput.m4:
    186-214,269-270); get = pread + in-place swap (ncmpio_getput.m4:415-470
    -> ncmpio_unpack_xbuf)."""
    from oracle import oracle as O
    lib = O.lib()
    lib.orc_c1_sequence.argtypes = [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    lib.orc_c1_sequence.restype = ctypes.c_int
    pm, gm = ctypes.c_double(0), (ctypes.c_double * 2)()
    rc = lib.orc_c1_sequence(path.encode(), var_offset, n, reps, ctypes.byref(pm), gm)
    put_ms, get_ms = pm.value, gm[0]
    xbytes = 4.0 * n
    out = {"unit": "GiB/s", "cores": 1, "kind": "port", "check_ok": rc == 0,
           "sample": f"the whole C1 request ({n} NC_INT, 4 MiB) on the same tmpfs file, median of {reps}: "
                     f"oracle restatement of the reference loop timed in C (oracle/ref_sequence.c), 1 thread: "
                     f"put = orc_in_swapn of the user buffer + pwrite + orc_in_swapn back; get = malloc xbuf + "
                     f"pread into it + orc_in_swapn + memcpy into the user buffer + free "
                     f"(ncmpio_getput.m4:415-427,468-470, ncmpio_util.c:884-888,934-936)"}
    if rc == 0:
        out.update({"value": round(2 * xbytes / ((put_ms + get_ms) * 1e-3) / GIB, 3),
                    "put_ms": round(put_ms, 4), "get_ms": round(get_ms, 4),
                    "get_ms_read_into_user_and_swap": round(gm[1], 4)})
    else:
        out["error"] = rc
    return out


C1_LEGS = (("host_8_io_threads", 0, None), ("host_1_io_thread", 0, "1"), ("device_buffers", 1, None))


def c1_first_order(reps):
    """Interleaved run order of the first-touch legs: the reference's
    sequence, then every library leg, `reps` times over, closing with the
    reference again -- so each library run has a reference run on both sides
    of it, and no leg always runs first."""
    order = []
    for k in range(reps):
        order.append("ref")
        legs = [name for name, _, _ in C1_LEGS]
        order += legs[k % len(legs):] + legs[:k % len(legs)]     # rotate which leg follows the reference
    return order + ["ref"]


def c1_first_compare(order, runs):
    """Per library run, its put/get/loop ratios against the mean of the two
    reference runs that bracket it in `order` (the nearest before and after).
    `runs` holds one result dict per entry of `order`."""
    for i, key in enumerate(order):
        r = runs[i]
        if key == "ref" or "put_ms" not in r:
            continue
        near = []
        for j in list(range(i - 1, -1, -1)) + list(range(i + 1, len(order))):
            if order[j] == "ref" and runs[j].get("check_ok") and (not near or (j > i) != (near[0] > i)):
                near.append(j)
            if len(near) == 2:
                break
        if not near:
            continue
        ref = {k: sum(runs[j][k] for j in near) / len(near) for k in ("put_ms", "get_ms", "put_loop_ms")}
        r["put_vs_reference"] = round(ref["put_ms"] / r["put_ms"], 3)
        r["get_vs_reference"] = round(ref["get_ms"] / r["get_ms"], 3)
        r["put_loop_vs_reference"] = round(ref["put_loop_ms"] / r["put_loop_ms"], 3)


def c1_first_touch(nrec=32, n=1 << 20, cpu=True, reps=2):
    """C1 under the reference's own benchmark pattern
    (benchmarks/C/pnetcdf_put_vara.c:193-209): a record variable x(time, n)
    NC_INT, each 4 MiB record put exactly once with ncmpi_put_vara_int_all
    (appended past the end of the file) and then got once
    (tests/mpi/api_check c1first, with PNCX_PHASES=1 for the per-phase
    host time of the puts and gets), per-call medians; beside it the
    reference's sequence on the same records (oracle/ref_sequence.c
    orc_c1_first_sequence: swap, pwrite, swap back, numrecs; malloc xbuf,
    pread, swap, memcpy, free).  The legs and the reference runs are
    interleaved (c1_first_order) and every library leg runs `reps` times;
    each run is compared with the reference runs on either side of it."""
    exe = os.path.join(ROOT, "tests", "mpi", "api_check")
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    path = os.path.join(shm, f"pncx_c1first_{os.getpid()}.nc")
    legs_by = {name: (dev, th) for name, dev, th in C1_LEGS}
    rec_offset = [None]

    def ref_run():
        from oracle import oracle as O
        lib = O.lib()
        lib.orc_c1_first_sequence.argtypes = [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_double)]
        lib.orc_c1_first_sequence.restype = ctypes.c_int
        if rec_offset[0] is None:               # the library's header length for this variable
            rec_offset[0] = lib_run("host_1_io_thread", probe=True).get("rec_offset")
        if rec_offset[0] is None:
            return {"check_ok": False, "error": "no record offset (the library's probe run failed)"}
        o = (ctypes.c_double * 6)()
        rc = lib.orc_c1_first_sequence(path.encode(), rec_offset[0], n, nrec, o)
        return {"check_ok": rc == 0, "error": rc} if rc else {
            "check_ok": True, "put_ms": round(o[0], 4), "get_ms": round(o[1], 4), "put_ms_min": round(o[2], 4),
            "get_ms_min": round(o[3], 4), "put_loop_ms": round(o[4], 3), "get_loop_ms": round(o[5], 3)}

    def lib_run(key, probe=False):
        dev, threads = legs_by[key]
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env["PNCX_PHASES"] = "1"
        if threads is not None:
            env["PNCX_IO_THREADS"] = threads
        r = subprocess.run([exe, "c1first", path, str(n), str(2 if probe else nrec), str(dev)],
                           capture_output=True, text=True, timeout=300, env=env)
        if r.returncode != 0:
            return {"error": r.returncode, "stderr": r.stderr[-400:]}
        o = json.loads(r.stdout.strip().splitlines()[-1])
        if probe:
            return o
        rec_offset[0] = o["rec_offset"]
        ph = o.get("put_phases", {})
        return {"put_ms": o["put_ms_median"], "get_ms": o["get_ms_median"], "put_ms_min": o["put_ms_min"],
                "get_ms_min": o["get_ms_min"], "put_loop_ms": o["put_loop_ms"], "get_loop_ms": o["get_loop_ms"],
                "close_ms": o["close_ms"], "errors": o["errors"],
                # the first put of the process and create..enddef, where the
                # library's one-time setup runs
                "put_first_ms": o.get("put_first_ms"), "get_first_ms": o.get("get_first_ms"),
                "create_to_enddef_ms": o.get("create_to_enddef_ms"),
                # us per put after the first, by phase (pncx_phase_name)
                "put_phases_us": {k.split(".", 1)[1]: v[0] for k, v in ph.items() if k.startswith("put.")},
                "put_phases": ph, "first_put_phases": o.get("first_put_phases"),
                "get_phases": o.get("get_phases")}

    order = [k for k in c1_first_order(reps) if cpu or k != "ref"]
    runs = []
    for key in order:
        runs.append(ref_run() if key == "ref" else lib_run(key))
    c1_first_compare(order, runs)
    out = {"pattern": f"benchmarks/C/pnetcdf_put_vara.c:193-209, one rank: record variable x(time, {n}) NC_INT, "
                      f"{nrec} records of 4 MiB each put once (appended) then got once; per-call medians",
           "loops": "put_loop_ms / get_loop_ms: the whole loops as the reference's benchmark times its write loop, "
                    "including the program's own update of each record's values (and, in device_buffers, its "
                    "4 MiB hipMemcpy of them to the device)",
           "order": order, "runs": runs}
    out["check_ok"] = all((r.get("check_ok") if k == "ref" else r.get("errors", 1) == 0)
                          for k, r in zip(order, runs))
    try:
        os.unlink(path)
    except OSError:
        pass
    return out


def c1_first_summary(ft):
    """The compact form of c1_first_touch's result for the printed line: per
    leg, every run's put/get medians, loop time and its ratios against the
    bracketing reference runs, and the put's phase means of the first run."""
    legs = {}
    for key, r in zip(ft["order"], ft["runs"]):
        name = "reference_sequence" if key == "ref" else key
        s = legs.setdefault(name, {})
        if "put_ms" not in r:
            s.setdefault("errors", []).append(r.get("error"))
            continue
        fields = ["put_ms", "get_ms", "put_loop_ms"]
        if key != "ref":
            fields += ["put_vs_reference", "get_vs_reference", "put_loop_vs_reference"]
        for f in fields:
            if f in r:
                s.setdefault(f, []).append(round(r[f], 3))
        if key != "ref" and "put_phases_us" in r and "put_phases_us" not in s:
            s["put_phases_us"] = {k: round(v) for k, v in r["put_phases_us"].items() if v >= 5}
    for name, s in legs.items():
        if s.get("put_ms"):
            s["put_ms_min_med_max"] = [min(s["put_ms"]), sorted(s["put_ms"])[len(s["put_ms"]) // 2], max(s["put_ms"])]
    return {"legs": legs, "check_ok": ft["check_ok"], "runs_in_order": " ".join(ft["order"])}


def c1_workload(cpu=True):
    res, path = c1_leg()
    out = {"unit": "GiB/s", "config": {
        "workload": "C1: benchmarks/C pattern, 1 MPI rank on tmpfs: 1-D 2^20 NC_INT ncmpi_put_vara_int_all + "
                    "ncmpi_get_vara_int_all through libpnetcdf.so",
        "elements": 1 << 20, "xtype": "NC_INT", "itype": "int", "file": "/dev/shm"},
        "note": "value = external bytes of one put + one get / (put_ms + get_ms), host buffers, 8 I/O threads; "
                "host-memory boundary: PCIe-bound, not an HBM roofline case (roofline null)",
        "roofline": None, "legs": res}
    h = res.get("host_8_io_threads", {})
    ok = all(isinstance(v, dict) and v.get("errors", 1) == 0 for k, v in res.items() if k != "var_offset")
    if "put_ms" in h:
        out["value"] = round(2 * 4.0 * (1 << 20) / ((h["put_ms"] + h["get_ms"]) * 1e-3) / GIB, 3)
        out["ms_per_step"] = round(h["put_ms"] + h["get_ms"], 4)
    if cpu and "var_offset" in res:
        out["cpu_baseline"] = c1_reference_sequence(path, res["var_offset"])
        ok = ok and out["cpu_baseline"]["check_ok"]
    try:
        os.unlink(path)
    except OSError:
        pass
    out["first_touch"] = c1_first_touch(cpu=cpu)
    out["check_ok"] = ok and out["first_touch"]["check_ok"]
    return out


# --------------------------------------------------------------- the printed line
DETAIL_PATH = os.path.join("profiles", "bench_detail_last.json")
LINE_MAX_CHARS = 6000          # the driver keeps the last ~8 KB of stdout+stderr


def _cpu_short(cb, head=True):
    if not isinstance(cb, dict):
        return cb
    return {k: cb[k] for k in (("value", "unit") if head else ("value",)) + ("cores", "kind", "put_ms", "get_ms")
            if k in cb}


def _roof_short(rf, head=True):
    if not isinstance(rf, dict):
        return rf
    keys = ("bound", "peak", "unit") if head else ()
    out = {k: rf[k] for k in keys + ("achieved", "frac", "traffic", "kernel", "kernel_ms_avg", "call_ms_avg")
           if k in rf}
    ts = rf.get("traffic_source")
    if isinstance(ts, dict):
        out["traffic_source"] = f"{ts.get('file')} round {ts.get('round')}"
    return out


def compact_line(full, detail_path=DETAIL_PATH):
    """The one JSON line rank 0 prints: the contract's keys and, per extra
    workload, its rate, roofline and CPU baseline -- everything else of the
    run (sample descriptions, C1's per-run phase breakdowns, rank lists) goes
    to `detail_path`, named in the line.  Kept under LINE_MAX_CHARS so the
    driver's captured tail holds every workload (BENCH_r05 lost C3 and C4 to
    a 10.8 KB line)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "slab_GiBps", "check_ok")
    line = {k: full[k] for k in keep if k in full}
    cfg = full.get("config", {})
    line["config"] = {k: cfg[k] for k in ("workload", "slab_gib_per_gpu", "elements_per_gpu", "records_per_gpu",
                                          "parallelism") if k in cfg}
    line["roofline"] = _roof_short(full.get("roofline"))
    line["cpu_baseline"] = _cpu_short(full.get("cpu_baseline"))
    if full.get("cpu_baseline_all_cores"):
        line["cpu_baseline_all_cores"] = _cpu_short(full["cpu_baseline_all_cores"])
    line["check"] = full.get("check", "")[:160]
    wls = {}
    for name, w in full.get("workloads", {}).items():
        if name == "c1":
            c = {k: w[k] for k in ("value", "unit", "ms_per_step", "check_ok") if k in w}
            h = w.get("legs", {})
            c["repeated_range"] = {k: {f: v[f] for f in ("put_ms", "get_ms") if f in v}
                                   for k, v in h.items() if isinstance(v, dict)}
            c["cpu_baseline"] = _cpu_short(w.get("cpu_baseline"), head=False)
            if "first_touch" in w:
                c["first_touch"] = c1_first_summary(w["first_touch"])
            wls[name] = c
            continue
        c = {k: w[k] for k in ("value", "ms_per_step", "steps", "n_gpus", "check_ok", "kernel_ms_per_rank")
             if k in w}
        c["roofline"] = _roof_short(w.get("roofline"), head=False)
        c["cpu_baseline"] = _cpu_short(w.get("cpu_baseline"), head=False)
        if w.get("cpu_baseline_all_cores"):
            c["cpu_baseline_all_cores"] = _cpu_short(w["cpu_baseline_all_cores"], head=False)
        wls[name] = c
    if wls:
        line["workloads"] = wls
    if "gather" in full:
        g = full["gather"]
        line["gather"] = {k: g[k] for k in ("collective", "bytes_per_rank", "chunks", "ms", "GBps_into_rank0",
                                            "checksums_ok", "via_xgmi") if k in g}
    if "ranks" in full:
        line["ranks"] = full["ranks"]
    line["detail"] = detail_path
    return line


def emit(full):
    """Write the whole result to DETAIL_PATH (best effort) and print the
    compact line."""
    try:
        with open(os.path.join(ROOT, DETAIL_PATH), "w") as f:
            json.dump(full, f, indent=1)
    except OSError:
        pass
    s = json.dumps(compact_line(full))
    print(s, flush=True)
    return s


def add_cpu_baselines(wls, budget):
    """1-core and 16-core oracle baselines beside the other 1-GPU configs
    (north_star: the reference's CPU swap/convert on the GPU box's own host
    cores in the same run; 16 = the host-core share of one GPU on the box)."""
    from oracle import oracle as O
    lib = O.lib()
    cores = min(16, os.cpu_count() or 1)
    if "c3" in wls:
        jobs, keep = cpu_c3_jobs(lib, seed=SEEDS["c3"])
        smp = "2^26 NC_INT -> double host sample in 16 slices (orc_getn)"
        wls["c3"]["cpu_baseline"] = cpu_baseline_jobs("c3", jobs, 1, budget, smp)
        wls["c3"]["cpu_baseline_all_cores"] = cpu_baseline_jobs("c3", jobs, cores, budget, smp)
        del jobs, keep
    for name, erange in (("c4", False), ("c4_erange", True)):
        if name not in wls:
            continue
        jobs, keep = cpu_c4_jobs(lib, erange, seed=SEEDS["c4"])
        smp = ("the whole C4 secondary workload in host memory: 128 float -> NC_SHORT (~18 % NC_ERANGE + fill) "
               "+ 128 NC_FLOAT putn of 2^20 elements" if erange else
               "the whole C4 workload in host memory: 128 NC_SHORT + 128 NC_FLOAT same-type putn of 2^20 elements")
        one = cpu_baseline_jobs(name, jobs, 1, budget, smp)
        allc = cpu_baseline_jobs(name, jobs, cores, budget, smp)
        targets = [name] + (["c4_async"] if name == "c4" and "c4_async" in wls else [])
        for t in targets:
            wls[t]["cpu_baseline"], wls[t]["cpu_baseline_all_cores"] = one, allc
        del jobs, keep


def device_identity(torch, local):
    """PCI domain:bus:device of this rank's GPU as one number (a float64
    holds it exactly), for the distinct-device check at N > 1."""
    p = torch.cuda.get_device_properties(local)
    dom, bus, dev = (int(getattr(p, k, -1)) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    if bus < 0:
        return float(local), f"local{local}"
    return float((dom << 16) | (bus << 8) | dev), f"{dom:04x}:{bus:02x}:{dev:02x}"


def worker(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("PNCX_DIST_BACKEND", "nccl")      # nccl == RCCL on ROCm
    if args.probe_launch:                                    # launcher check: no GPU work at all
        print(json.dumps({"rank": rank, "world": world, "local_rank": local, "gpus_arg": args.gpus}), flush=True)
        return 0
    if backend != "nccl":
        local = 0          # rehearsal: every rank on GPU 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:   # rehearsal of the N>1 path with several ranks on one GPU
            dist.init_process_group(backend)
    from pnetcdf_amd import pncx
    from pnetcdf_amd.shard import Group
    lib = pncx.lib()
    group = Group(dist, torch.device("cuda", local) if backend == "nccl" else "cpu")
    stream = torch.cuda.current_stream()
    sptr = ctypes.c_void_p(stream.cuda_stream)
    ranks = None
    if world > 1:
        # one process per GPU: every rank's GPU must be a different device
        # (PCI address gathered over the group); the gloo rehearsal puts
        # every rank on GPU 0 on purpose and says so
        ident, name = device_identity(torch, local)
        ids = [r[0] for r in group.all_gather_floats([ident])]
        distinct = len(set(ids)) == world
        ranks = {"backend": "rccl" if backend == "nccl" else backend, "world_size": world,
                 "local_device_of_rank0": name, "distinct_devices": distinct,
                 "pci_of_ranks": ["%04x:%02x:%02x" % ((int(i) >> 16), (int(i) >> 8) & 0xFF, int(i) & 0xFF)
                                  for i in ids]}
        if backend == "nccl":
            ranks["rccl_world_size"] = dist.get_world_size()
            if not distinct:
                if rank == 0:
                    print(f"bench.py: ranks share GPUs {ranks['pci_of_ranks']}; refusing to report a "
                          f"{world}-GPU number", file=sys.stderr)
                return 2

    # ------------------------------------------------ headline (value)
    head = "c4" if args.workload == "c4_async" else args.workload
    if args.workload == "c4_async":
        args.async_batch = True
    wl = make_workload(args.workload if args.workload != "c4_async" else "c4", torch, lib, sptr, args, world, rank)
    elapsed, kern_ms, call_ms = measure(torch, lib, group, stream, wl, args.steps, args.warmup)
    ok = group.all_true(wl.check())
    value, ms_per_step, roof = summary(wl, elapsed, kern_ms, call_ms, args.steps, world)
    if ranks is not None:
        ranks["kernel_ms_per_rank"] = [round(r[0], 4) for r in group.all_gather_floats([wl.rank_kernel_ms])]
    gather = None
    if world > 1 and args.gather_gib > 0 and head == "c2":
        gib = args.gather_gib if backend == "nccl" else min(args.gather_gib, 1.0)   # gloo rehearsal: 1 GiB
        gather = gather_leg(torch, group, wl._tbuf, gib, min(args.gather_chunk_gib, gib), to_cpu=backend != "nccl")
    line = {
        "metric": "GiB/s device-resident swap+type-convert, 2/4/8-byte NC arrays",
        "value": round(value, 2),
        "slab_GiBps": round(value * wl.slab_per_elem / wl.bytes_per_elem, 2),   # external bytes / t
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": wl.dtype,
        "data": "synthetic (splitmix64 bit patterns generated on the GPU)",
        "config": wl.cfg,
        "roofline": roof,
        "check_ok": ok,
        "check": wl.check_desc + (" (on every rank, AND-reduced)" if world > 1 else ""),
    }
    wl.free()
    del wl
    torch.cuda.empty_cache()

    # ------------------------------------------------ the other configs
    # C3 and C4 run at every N: each rank converts its own copy of the
    # workload (the reference's decomposition: per-rank subarrays with no
    # communication in the conversion, ncmpio_i_getput.m4:332,416), timed
    # between barriers with the max over ranks, checks AND-reduced; value =
    # the bytes of all ranks / that time.  C1 is the one-rank file case.
    if not args.no_extra and head == "c2":
        extra = {}
        for name in EXTRA:
            w = make_workload(name, torch, lib, sptr, args, world, rank)
            el, km, cm = measure(torch, lib, group, stream, w, args.extra_steps, max(args.warmup, args.extra_warmup))
            v, mps, rf = summary(w, el, km, cm, args.extra_steps, world)
            extra[name] = {"value": round(v, 2), "unit": "GiB/s", "ms_per_step": round(mps, 4),
                           "steps": args.extra_steps, "n_gpus": world, "scaling": "weak", "dtype": w.dtype,
                           "config": w.cfg, "roofline": rf, "check_ok": group.all_true(w.check()),
                           "check": w.check_desc + (" (on every rank, AND-reduced)" if world > 1 else "")}
            if world > 1:
                extra[name]["kernel_ms_per_rank"] = [round(r[0], 4) for r in
                                                     group.all_gather_floats([w.rank_kernel_ms])]
            w.free()
            del w
            torch.cuda.empty_cache()
        if world == 1 and not args.no_c1:
            extra["c1"] = c1_workload(cpu=rank == 0 and not args.no_cpu_baseline)
        line["workloads"] = extra

    if rank == 0:
        if world == 1 and not args.no_cpu_baseline and head == "c2":
            line["cpu_baseline"] = cpu_baseline_swap8(args.cpu_budget)
            line["cpu_baseline_all_cores"] = cpu_baseline_swap8_threads()
            if "workloads" in line:
                add_cpu_baselines(line["workloads"], args.cpu_budget_extra)
        else:
            line["cpu_baseline"] = None
        if gather is not None:
            line["gather"] = gather
        if ranks is not None:
            line["ranks"] = ranks
        emit(line)
    if dist is not None:
        dist.destroy_process_group()
    return 0


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c4_async", "c4_erange"])
    ap.add_argument("--slab-gib", type=float, default=32.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="N=1, c2: skip the c3/c4/c1 workloads")
    ap.add_argument("--no-c1", action="store_true", help="N=1, c2: skip the c1 file-level leg")
    ap.add_argument("--extra-steps", type=int, default=200,
                    help="timed calls of each extra workload (20 calls of ~0.25 ms read 2-5 %% high: the rate settles "
                         "over the first ~100, profiles/r02s_bench_x200.json)")
    ap.add_argument("--extra-warmup", type=int, default=20,
                    help="untimed calls before each extra workload's timed ones (the first ~20 batch calls "
                         "after its buffers are made run 1-3 %% slower, tools/c4_ab.py round 0)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--cpu-budget-extra", type=float, default=3.0,
                    help="seconds of each 1-core / all-core CPU baseline of the c3/c4 workloads")
    ap.add_argument("--async-batch", action="store_true",
                    help="c4: pncx_dev_batch_async (statuses stay in HBM, calls queue back to back) "
                         "instead of the synchronous pncx_dev_batch")
    ap.add_argument("--gather-gib", type=float, default=32.0,
                    help="N>1, c2: GiB per rank gathered into rank 0 after the timed region (0 = off)")
    ap.add_argument("--gather-chunk-gib", type=float, default=2.0)
    ap.add_argument("--probe-launch", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            return launch_ranks(args.gpus, argv)
    elif int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}; refusing to report a mislabelled run",
              file=sys.stderr)
        return 2
    return worker(args)


if __name__ == "__main__":
    sys.exit(main())
