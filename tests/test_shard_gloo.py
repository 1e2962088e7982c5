"""The N>1 path (config 5 record sharding) with world_size 2 over gloo (CPU).

Each rank converts its record slab of a small NC_DOUBLE record variable
(the CPU oracle stands in for the per-GPU kernel here: this test covers the
partition and the control collectives, the kernels are covered on the GPU),
then the slabs are gathered and compared with a whole-variable conversion.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pnetcdf_amd.shard import Group, record_extent, record_slab


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_record_slab_partition():
    for nrecs in (0, 1, 7, 256, 257):
        for world in (1, 2, 3, 8):
            got = [record_slab(nrecs, world, r) for r in range(world)]
            assert sum(c for _, c in got) == nrecs
            pos = 0
            for first, count in got:
                assert first == pos
                pos += count
            assert max(c for _, c in got) - min(c for _, c in got) <= 1
    assert record_extent(1024, 1 << 30, 32, 32) == (1024 + 32 * (1 << 30), 1024 + 64 * (1 << 30))
    with pytest.raises(ValueError):
        record_slab(8, 2, 2)


def _worker(rank, world, port, nrecs, per_rec, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from pnetcdf_amd import nctypes as T
        g = Group(dist, "cpu")
        rng = np.random.default_rng(0x5EED0005)
        whole = rng.standard_normal(nrecs * per_rec) * 1e3
        whole[5] = 1e300                        # one out-of-range element (for NC_FLOAT)
        first, count = record_slab(nrecs, world, rank)
        mine = whole[first * per_rec:(first + count) * per_rec]
        xb, st = O.putn(5, T.NC_FLOAT, mine, T.ITYPE_DOUBLE, fill=T.fill_bytes(T.NC_FLOAT))
        g.barrier()
        tmax = g.max([float(rank + 1), 2.0 * rank])
        err = g.first_error(st)
        buf = torch.from_numpy(np.frombuffer(xb, np.uint8).copy())
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([buf.numel()]))
        mx = max(int(s.item()) for s in sizes)
        pad = torch.zeros(mx, dtype=torch.uint8)
        pad[:buf.numel()] = buf
        parts = [torch.zeros(mx, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, pad)
        if rank == 0:
            joined = b"".join(p[:int(s.item())].numpy().tobytes() for p, s in zip(parts, sizes))
            ref, st_ref = O.putn(5, T.NC_FLOAT, whole, T.ITYPE_DOUBLE, fill=T.fill_bytes(T.NC_FLOAT))
            out_q.put((joined == ref, err, st_ref, tmax))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("nrecs", [8, 9])
def test_sharded_records_gloo(nrecs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, nrecs, 1000, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    same, err, st_ref, tmax = q.get(timeout=10)
    assert same                      # the slabs tile the variable exactly
    assert err == st_ref == -60      # first error propagates from the rank that saw it
    assert tmax == [2.0, 2.0]        # max over ranks


def _gather_worker(rank, world, port, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = Group(dist, "cpu")
        # each rank's converted record slab (bit patterns), as bench.py's gather leg sends it
        mine = torch.from_numpy(np.random.default_rng(100 + rank).integers(-2**62, 2**62, 4096, dtype=np.int64))
        sums = g.all_gather_int(int(mine.sum().item()))
        got = g.gather_slices(mine)
        if rank == 0:
            ok = len(got) == world and all(int(t.sum().item()) == s for t, s in zip(got, sums))
            exp = [np.random.default_rng(100 + r).integers(-2**62, 2**62, 4096, dtype=np.int64) for r in range(world)]
            ok = ok and all(np.array_equal(t.numpy(), e) for t, e in zip(got, exp))
            out_q.put(ok)
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_gather_into_rank0_gloo():
    """config 5's optional exchange (bench.py gather leg): slabs gathered into
    rank 0 arrive intact and match the senders' checksums"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def _file_worker(rank, world, port, path, nrecs, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pnetcdf_amd import ncfile as N
        from pnetcdf_amd import nctypes as T
        g = Group(dist, "cpu")
        if rank == 0:                                   # rank 0 defines the file (the header writer)
            err, ncid = N.create(path, N.NC_64BIT_DATA)
            N.def_dim(ncid, "time", N.NC_UNLIMITED)
            N.def_dim(ncid, "x", 64)
            N.def_var(ncid, "v", T.NC_BYTE, [0, 1])
            assert N.enddef(ncid) == 0 and N.close(ncid) == 0
        g.barrier()
        err, ncid = N.open(path, N.NC_WRITE)
        assert err == 0
        first, count = record_slab(nrecs, world, world - 1 - rank)   # rank 0 holds the LAST records
        recs = np.stack([np.full(64, (r * 7) % 127, np.int8) for r in range(first, first + count)])
        assert N.put_var(ncid, 0, recs, [first, 0], [count, 64]) == 0
        mine = N.inq_dim(ncid, 0)[2]
        numrecs = int(g.max([float(mine)])[0])          # ncmpio_sync_numrecs: MAX over ranks
        if rank == 0:
            assert N.sync_numrecs(ncid, numrecs) == 0
        g.barrier()
        assert N.close(ncid) == 0                       # rank 1 (fewer records) must not lower numrecs
        g.barrier()
        if rank == 0:
            err, ncid = N.open(path)
            ok = N.inq_dim(ncid, 0)[2] == nrecs
            out = np.zeros((nrecs, 64), np.int8)
            ok = ok and N.get_var(ncid, 0, out) == 0
            ok = ok and all(np.all(out[r] == (r * 7) % 127) for r in range(nrecs))
            N.close(ncid)
            out_q.put(bool(ok))
    finally:
        dist.destroy_process_group()


def test_two_ranks_write_disjoint_records_gloo(tmp_path):
    """config 5 at file level: each rank writes its record slab of one file,
    numrecs reduced with MAX and recorded by rank 0"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "shared.nc")
    procs = [ctx.Process(target=_file_worker, args=(r, 2, port, path, 9, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True
