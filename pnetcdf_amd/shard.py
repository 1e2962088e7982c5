"""Record-slab sharding of a request across the GPUs of one node (config 5).

A record variable's records are independent and, for a single record
variable, contiguous in the file (record r starts at begin + r*recsize with
recsize = the record's own size, ncmpio_enddef.c:586-607).  The reference
splits a record request into per-record sub-requests
(ncmpio_i_getput.m4:332,416); here each rank (one GPU) takes one contiguous
slab of records and converts it with no data-path communication.  The only
exchanges are control: a barrier around the timed region, the max of the
per-rank times, and the "first error" of the conversions (NC_ERANGE is the
only error a conversion produces, so the minimum status over ranks is the
reference's first-error semantics, ncx.m4:2487-2488).

The one data exchange is optional and reported apart from the conversion
rate: gathering converted records into one GPU over xGMI
(`gather_slices`, RCCL gather of device tensors) for the config-5 variant
that hands the whole variable to a single consumer.

The same helpers run over RCCL (backend "nccl", device tensors) in bench.py
and over gloo (CPU tensors) in tests/test_shard_gloo.py.
"""


def record_slab(nrecs, world, rank):
    """Balanced contiguous partition of nrecs records: (first, count)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    base, rem = divmod(nrecs, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)


def record_extent(begin, recsize, first, count):
    """Byte range [start, end) of records first..first+count-1 of a single
    record variable in the file."""
    return begin + first * recsize, begin + (first + count) * recsize


class Group:
    """Control-plane collectives for the sharded run (no data movement)."""

    def __init__(self, dist=None, device="cpu"):
        self.dist = dist
        self.device = device

    @property
    def world(self):
        return self.dist.get_world_size() if self.dist is not None else 1

    @property
    def rank(self):
        return self.dist.get_rank() if self.dist is not None else 0

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, values):
        """Element-wise max over ranks of a list of floats."""
        if self.dist is None:
            return list(values)
        import torch
        t = torch.tensor(list(values), dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return [float(v) for v in t.cpu()]

    def sum(self, values):
        if self.dist is None:
            return list(values)
        import torch
        t = torch.tensor(list(values), dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return [float(v) for v in t.cpu()]

    def gather_slices(self, t, to_cpu=False):
        """Gather one equal-size tensor per rank into rank 0 (dist.gather:
        RCCL over xGMI for device tensors).  Returns the per-rank list on
        rank 0 and None elsewhere."""
        if self.dist is None:
            return [t]
        src = t.cpu() if to_cpu else t
        lst = [src.new_empty(src.shape) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(src, gather_list=lst, dst=0)
        return lst

    def all_gather_int(self, value):
        """int64 value of every rank, on every rank (checksums)."""
        if self.dist is None:
            return [int(value)]
        import torch
        t = torch.tensor([int(value)], dtype=torch.int64, device=self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    def all_gather_floats(self, values):
        """Every rank's list of floats (equal lengths), on every rank:
        [[rank 0's values], [rank 1's], ...]."""
        if self.dist is None:
            return [list(values)]
        import torch
        t = torch.tensor(list(values), dtype=torch.float64, device=self.device)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [[float(v) for v in o.cpu()] for o in out]

    def all_true(self, flag):
        """True on every rank iff flag holds on every rank."""
        return self.max([0.0 if flag else 1.0])[0] == 0.0

    def first_error(self, status):
        """min over ranks of an NC status (0 = NC_NOERR, negatives = errors)."""
        if self.dist is None:
            return int(status)
        import torch
        t = torch.tensor([int(status)], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return int(t.item())
