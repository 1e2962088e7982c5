"""Randomised operation sequences through the file layer against a model
(test infrastructure for tests/test_gpu_file_fuzz.py and
tests/test_file_fuzz_cpu.py).

A file with a handful of fixed-size and record variables is created in
NC_FILL mode; then a seeded stream of operations runs against it: blocking
and nonblocking puts and gets (vara, vars with strides, varm with permuted
and gapped imaps), from host numpy buffers and from device tensors, with
every internal type the external type admits, values that are sometimes out
of range.  The model keeps each variable's external (big-endian) bytes and
which elements are known; the expected bytes of a put and the expected
values of a get come from the CPU oracle's putn / getn (the reference's
ncx conversions, oracle/), applied at the file positions the request
selects.  Gets are compared element by element where the model knows the
bytes, user-buffer positions a varm does not map must keep their sentinel,
statuses must match (NC_ERANGE where the oracle reports it), and after
close the file's bytes are compared with the model through the independent
header parser (tests/cdfparse.py).

The reference has no such fuzz; its file-level tests (test/testcases/
flexible*.c, test_vard*.c, ivarn.c, tst_def_var_fill.c ...) each fix one
layout.  This drives the same entry points through many layouts at once.
"""
import os

import numpy as np

from pnetcdf_amd import nctypes as T
from tests import cdfparse

NUMERIC_ITYPES = [T.ITYPE_SCHAR, T.ITYPE_UCHAR, T.ITYPE_SHORT, T.ITYPE_USHORT, T.ITYPE_INT, T.ITYPE_UINT,
                  T.ITYPE_LONG, T.ITYPE_FLOAT, T.ITYPE_DOUBLE, T.ITYPE_LONGLONG, T.ITYPE_ULONGLONG]
CDF5_XTYPES = [T.NC_BYTE, T.NC_SHORT, T.NC_INT, T.NC_FLOAT, T.NC_DOUBLE, T.NC_UBYTE, T.NC_USHORT, T.NC_UINT,
               T.NC_INT64, T.NC_UINT64]
CLASSIC_XTYPES = [T.NC_BYTE, T.NC_SHORT, T.NC_INT, T.NC_FLOAT, T.NC_DOUBLE]
SAME_ITYPE = {T.NC_BYTE: T.ITYPE_SCHAR, T.NC_SHORT: T.ITYPE_SHORT, T.NC_INT: T.ITYPE_INT,
              T.NC_FLOAT: T.ITYPE_FLOAT, T.NC_DOUBLE: T.ITYPE_DOUBLE, T.NC_UBYTE: T.ITYPE_UCHAR,
              T.NC_USHORT: T.ITYPE_USHORT, T.NC_UINT: T.ITYPE_UINT, T.NC_INT64: T.ITYPE_LONGLONG,
              T.NC_UINT64: T.ITYPE_ULONGLONG, T.NC_CHAR: T.ITYPE_CHAR}
SENTINEL = 0x5A


class Var:
    def __init__(self, varid, name, xtype, shape, is_rec):
        self.varid, self.name, self.xtype, self.shape, self.is_rec = varid, name, xtype, list(shape), is_rec
        self.xs = T.xlen(xtype)
        self.per = int(np.prod(self.shape[1:] if is_rec else self.shape, dtype=np.int64))   # elements per record / in all
        self.fixed = None        # fixed: uint8 bytes of the whole variable
        self.fknown = None
        self.recs = {}           # record: r -> (uint8 bytes, bool known)

    def record(self, r):
        if r not in self.recs:
            self.recs[r] = (np.zeros(self.per * self.xs, np.uint8), np.zeros(self.per, bool))
        return self.recs[r]


class TorchDev:
    """device buffers from torch (hipMalloc'ed HBM)"""

    def __init__(self, torch):
        self.torch = torch

    def alloc(self, arr):
        t = self.torch.from_numpy(arr.view(np.uint8).copy()).cuda()
        return t, t.data_ptr()

    def download(self, t, arr):
        self.torch.cuda.synchronize()
        arr.view(np.uint8)[:] = t.cpu().numpy()

    def stream(self):
        return self.torch.cuda.current_stream().cuda_stream

    def free(self, t):
        pass

    def sync(self):
        self.torch.cuda.synchronize()


class StandinDev:
    """device buffers from the CPU stand-in of a test build (tools/tsan/).
    itypes: only these internal types take device buffers (None: all)"""

    def __init__(self, lib, itypes=None):
        import ctypes
        self.ct, self.lib, self.itypes = ctypes, lib, itypes
        lib.pncxrt_malloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        lib.pncxrt_free.argtypes = [ctypes.c_void_p]
        lib.pncxrt_stream_sync.argtypes = [ctypes.c_void_p]

    def alloc(self, arr):
        p = self.ct.c_void_p()
        assert self.lib.pncxrt_malloc(self.ct.byref(p), max(arr.nbytes, 1)) == 0
        self.ct.memmove(p.value, arr.ctypes.data, arr.nbytes)
        return p, p.value

    def download(self, h, arr):
        self.lib.pncxrt_stream_sync(None)
        self.ct.memmove(arr.ctypes.data, h.value, arr.nbytes)
        self.lib.pncxrt_free(h)

    def stream(self):
        return None

    def free(self, h):
        self.lib.pncxrt_free(h)

    def sync(self):
        self.lib.pncxrt_stream_sync(None)


class FileFuzz:
    """One file, one seed.  conv: the oracle adapter (tests/converters.py
    OracleConv).  same_type: only the internal type equal to the external
    one (no conversion: what the synchronous CPU stand-in carries out).
    torch: the torch module (device buffers through TorchDev), or dev: a
    StandinDev (the CPU stand-ins of tools/tsan/), or neither.  imap: varm requests (the
    stand-in has no gather kernel).  big: one variable of 1-2 Mi elements."""

    def __init__(self, path, seed, conv, fmt=5, same_type=False, torch=None, big=True, imap=True, dev=None):
        from pnetcdf_amd import ncfile as N
        self.N, self.path, self.conv, self.fmt = N, path, conv, fmt
        self.rng = np.random.default_rng(seed)
        self.same_type, self.big, self.use_imap = same_type, big, imap
        self.dev = dev if dev is not None else (TorchDev(torch) if torch is not None else None)
        self.vars = []
        self.numrecs = 0
        self.pending = {}        # varid -> (kind, request id, check closure)
        self.counts = {}
        self.log = []            # one line per operation, for a failing seed

    # ------------------------------------------------------------ schema
    def create(self):
        N, rng = self.N, self.rng
        cmode = {1: 0, 2: N.NC_64BIT_OFFSET, 5: N.NC_64BIT_DATA}[self.fmt]
        err, self.ncid = N.create(self.path, cmode)
        assert err == 0, err
        assert N.set_fill(self.ncid, N.NC_FILL)[0] == 0
        dims = [N.def_dim(self.ncid, "t", N.NC_UNLIMITED)[1]]
        lens = [int(rng.integers(1, 9)), int(rng.integers(3, 40)), int(rng.integers(2, 70)), int(rng.integers(1, 5))]
        for k, n in enumerate(lens):
            dims.append(N.def_dim(self.ncid, f"d{k}", n)[1])
        xts = CDF5_XTYPES if self.fmt == 5 else CLASSIC_XTYPES
        nvars = int(rng.integers(4, 8))
        for i in range(nvars):
            xt = int(rng.choice(xts))
            is_rec = bool(rng.random() < 0.4)
            nd = int(rng.integers(1, 4))
            pick = [int(x) for x in rng.choice(len(lens), size=nd - (1 if is_rec else 0), replace=True)]
            shape = ([0] if is_rec else []) + [lens[p] for p in pick]
            dimids = ([dims[0]] if is_rec else []) + [dims[p + 1] for p in pick]
            err, vid = N.def_var(self.ncid, f"v{i}", xt, dimids)
            assert err == 0, err
            self.vars.append(Var(vid, f"v{i}", xt, shape, is_rec))
        if self.big:         # one variable past a staging slot's worth of chunks
            n = int(rng.integers(1, 3)) * (1 << 20) + int(rng.integers(0, 4096))
            xt = int(rng.choice([T.NC_INT, T.NC_DOUBLE, T.NC_SHORT, T.NC_FLOAT]))
            dbig = N.def_dim(self.ncid, "big", n)[1]
            err, vid = N.def_var(self.ncid, "vbig", xt, [dbig])
            assert err == 0
            self.vars.append(Var(vid, "vbig", xt, [n], False))
        assert N.enddef(self.ncid) == 0
        # NC_FILL: fixed-size variables hold the fill value from enddef on
        for v in self.vars:
            if not v.is_rec:
                fb = np.frombuffer(T.fill_bytes(v.xtype), np.uint8)[::-1]        # big-endian
                v.fixed = np.tile(fb, v.per).copy()
                v.fknown = np.ones(v.per, bool)

    # ------------------------------------------------------------ helpers
    def _itype(self, v):
        if v.xtype == T.NC_CHAR or self.same_type:
            return SAME_ITYPE[v.xtype]
        return int(self.rng.choice(NUMERIC_ITYPES))

    def _values(self, itype, xtype, n):
        rng = self.rng
        dt = np.dtype(T.ITYPE_NP[itype])
        wide = rng.random() < 0.25                     # full range of the internal type: NC_ERANGE likely
        if dt.kind == "f":
            if wide:
                v = rng.standard_normal(n) * 10.0 ** rng.integers(0, 30)
                if rng.random() < 0.3 and n:
                    v[rng.integers(0, n)] = np.nan
            else:
                lo, hi = self._xrange(xtype)
                v = rng.uniform(max(lo, -1e6), min(hi, 1e6), n)
                if np.dtype(T.XTYPE_NP[xtype]).kind != "f":
                    v = np.trunc(v)
            return v.astype(dt)
        info = np.iinfo(dt)
        if wide:
            return rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        lo, hi = self._xrange(xtype)
        lo, hi = max(int(lo), info.min), min(int(hi), info.max)
        return rng.integers(lo, hi, n, dtype=np.int64 if hi < 2 ** 63 else np.uint64, endpoint=True).astype(dt)

    @staticmethod
    def _xrange(xtype):
        d = np.dtype(T.XTYPE_NP[xtype])
        if d.kind == "f":
            return (-3.0e38, 3.0e38) if d.itemsize == 4 else (-1e300, 1e300)
        i = np.iinfo(d)
        return i.min, i.max

    def _request(self, v, write):
        """start, count, stride (or None), imap (or None) and the file element
        index of each selected element in C order over count"""
        rng = self.rng
        nd = len(v.shape)
        start, count, stride = [], [], []
        for d in range(nd):
            if v.is_rec and d == 0:
                top = self.numrecs + (2 if write else 0)
                if top == 0:
                    return None
                s = int(rng.integers(0, top))
                st = int(rng.integers(1, 3))
                c = int(rng.integers(1, min(3, (top - 1 - s) // st + 1) + 1))
            else:
                n = v.shape[d]
                big = v.name == "vbig"
                s = int(rng.integers(0, n)) if not big or rng.random() < 0.5 else 0
                st = 1 if big and rng.random() < 0.7 else int(rng.choice([1, 1, 1, 2, 3]))
                cmax = (n - 1 - s) // st + 1
                c = int(rng.integers(1, cmax + 1)) if not (big and rng.random() < 0.5) else cmax
            start.append(s)
            count.append(c)
            stride.append(st)
        use_stride = any(x != 1 for x in stride)
        # file element indices (record, within-record element) in C order over count
        grids = np.meshgrid(*[s + np.arange(c) * st for s, c, st in zip(start, count, stride)], indexing="ij")
        pos = [g.reshape(-1) for g in grids]
        if v.is_rec:
            rec = pos[0]
            inner = np.zeros_like(rec)
            for d in range(1, nd):
                inner = inner * v.shape[d] + pos[d]
        else:
            rec = None
            inner = np.zeros(pos[0].shape, np.int64)
            for d in range(nd):
                inner = inner * v.shape[d] + pos[d]
        imap = None
        if self.use_imap and rng.random() < 0.3 and v.name != "vbig":
            # a permuted, possibly gapped user layout: dims in random order, each
            # extent padded by 0..2 elements
            order = list(rng.permutation(nd))
            imap = [0] * nd
            step = 1
            for d in reversed(order):
                imap[d] = step
                step *= count[d] + int(rng.integers(0, 3))
        return dict(start=start, count=count, stride=stride if use_stride else None, imap=imap,
                    rec=rec, inner=inner, n=int(np.prod(count)))

    @staticmethod
    def _buf_offsets(req):
        """user-buffer element offset of each selected element (C order over count)"""
        count, imap = req["count"], req["imap"]
        if imap is None:
            return np.arange(req["n"], dtype=np.int64)
        grids = np.meshgrid(*[np.arange(c) * m for c, m in zip(count, imap)], indexing="ij")
        return sum(g.reshape(-1) for g in grids).astype(np.int64)

    def _model_bytes(self, v, req):
        """(bytes in C order over count, known mask)"""
        xs = v.xs
        out = np.zeros(req["n"] * xs, np.uint8)
        known = np.zeros(req["n"], bool)
        if v.is_rec:
            for r in np.unique(req["rec"]):
                sel = np.nonzero(req["rec"] == r)[0]
                if int(r) not in v.recs:
                    continue
                b, k = v.recs[int(r)]
                e = req["inner"][sel]
                out.reshape(-1, xs)[sel] = b.reshape(-1, xs)[e]
                known[sel] = k[e]
        else:
            e = req["inner"]
            out.reshape(-1, xs)[:] = v.fixed.reshape(-1, xs)[e]
            known[:] = v.fknown[e]
        return out, known

    def _apply(self, v, req, xbytes):
        xs = v.xs
        xb = np.frombuffer(xbytes, np.uint8).reshape(-1, xs)
        if v.is_rec:
            for r in np.unique(req["rec"]):
                sel = np.nonzero(req["rec"] == r)[0]
                b, k = v.record(int(r))
                e = req["inner"][sel]
                b.reshape(-1, xs)[e] = xb[sel]
                k[e] = True
            self.numrecs = max(self.numrecs, int(req["rec"].max()) + 1)
        else:
            v.fixed.reshape(-1, xs)[req["inner"]] = xb
            v.fknown[req["inner"]] = True

    def _fill(self, v):
        return T.fill_bytes(v.xtype)

    def _count(self, what, v=None, it=None, req=None, err=None):
        self.counts[what] = self.counts.get(what, 0) + 1
        if v is not None:
            self.log.append(f"{what} {v.name} x{v.xtype} {T.INAME[it]} start={req['start']} count={req['count']} "
                            f"stride={req['stride']} imap={req['imap']} err={err} numrecs={self.numrecs}")

    # ------------------------------------------------------------ operations
    def _dev_ok(self, itype):
        return self.dev is not None and (getattr(self.dev, "itypes", None) is None or itype in self.dev.itypes)

    def _dev_call(self, name, v, req, ptr, it):
        import ctypes
        keep, a = self.N._args(req["start"], req["count"], req["stride"], req["imap"])
        return getattr(self.N.lib(), name)(self.ncid, v.varid, *a, ptr, it, ctypes.c_void_p(self.dev.stream()))

    def put(self, v, nonblocking):
        N, rng = self.N, self.rng
        req = self._request(v, True)
        if req is None:
            return
        it = self._itype(v)
        vals = self._values(it, v.xtype, req["n"])
        offs = self._buf_offsets(req)
        blen = int(offs.max()) + 1 if req["n"] else 0
        buf = np.zeros(blen, T.ITYPE_NP[it])
        buf[offs] = vals
        exp, st = self.conv.putn(self.fmt, v.xtype, vals, it, self._fill(v))
        dev = not nonblocking and req["imap"] is None and self._dev_ok(it) and rng.random() < 0.4
        args = (req["start"], req["count"], req["stride"], req["imap"])
        if dev:
            h, ptr = self.dev.alloc(buf)
            err = self._dev_call("pncx_nc_put_varm_dev", v, req, ptr, it)
            self.dev.sync()
            self.dev.free(h)
            self._count("put_dev", v, it, req, err)
        elif nonblocking:
            err, rid = N.iput_var(self.ncid, v.varid, buf, *args, itype=it)
            assert err == 0, ("iput", err)
            self.pending[v.varid] = ("put", rid, buf, st, lambda: self._apply(v, req, exp))
            self._count("iput", v, it, req, err)
            return
        else:
            err = N.put_var(self.ncid, v.varid, buf, *args, itype=it)
            self._count("put", v, it, req, err)
        assert err == st, ("put", v.name, T.INAME[it], req["start"], req["count"], req["stride"], req["imap"], err, st)
        self._apply(v, req, exp)

    def get(self, v, nonblocking):
        N, rng = self.N, self.rng
        req = self._request(v, False)
        if req is None:
            return
        it = self._itype(v)
        offs = self._buf_offsets(req)
        blen = int(offs.max()) + 1 if req["n"] else 0
        xb, known = self._model_bytes(v, req)
        exp, st = self.conv.getn(self.fmt, v.xtype, xb.tobytes(), it)
        args = (req["start"], req["count"], req["stride"], req["imap"])
        out = np.full(blen * T.ilen(it), SENTINEL, np.uint8).view(T.ITYPE_NP[it])
        dev = not nonblocking and req["imap"] is None and self._dev_ok(it) and rng.random() < 0.4

        def check(err):
            if known.all():
                assert err == st, ("get status", v.name, T.INAME[it], req["start"], req["count"], err, st)
            else:
                assert err in (0, T.NC_ERANGE), err
            got = out[offs]
            ok = (got.view(np.uint8).reshape(-1, T.ilen(it)) == exp.view(np.uint8).reshape(-1, T.ilen(it))).all(1)
            bad = np.nonzero(known & ~ok)[0]
            assert bad.size == 0, ("get values", v.name, T.INAME[it], req["start"], req["count"], req["stride"],
                                   req["imap"], int(bad[0]), got[bad[0]], exp[bad[0]])
            if req["imap"] is not None:          # positions the imap does not map keep the sentinel
                rest = np.ones(blen, bool)
                rest[offs] = False
                assert (out.view(np.uint8).reshape(-1, T.ilen(it))[rest] == SENTINEL).all(), "get wrote outside its map"

        if dev:
            h, ptr = self.dev.alloc(out)
            err = self._dev_call("pncx_nc_get_varm_dev", v, req, ptr, it)
            self.dev.download(h, out)
            self._count("get_dev", v, it, req, err)
        elif nonblocking:
            err, rid = N.iget_var(self.ncid, v.varid, out, *args, itype=it)
            assert err == 0, ("iget", err)
            self.pending[v.varid] = ("get", rid, out, None, check)
            self._count("iget", v, it, req, err)
            return
        else:
            err = N.get_var(self.ncid, v.varid, out, *args, itype=it)
            self._count("get", v, it, req, err)
        check(err)

    def wait(self):
        if not self.pending:
            return
        items = list(self.pending.values())
        err, sts = self.N.wait_all(self.ncid, [p[1] for p in items])
        assert err in (0, T.NC_ERANGE), err
        for (kind, _rid, _buf, st, fin), s in zip(items, sts):
            if kind == "put":
                assert s == st, ("iput status", s, st)
                fin()
            else:
                fin(s)
        self.pending.clear()
        self._count("wait")
        self.log.append("wait")

    def step(self):
        rng = self.rng
        v = self.vars[int(rng.integers(0, len(self.vars)))]
        if v.varid in self.pending or (v.is_rec and self.pending and rng.random() < 0.5):
            self.wait()                     # one request per variable; numrecs settles before record gets
        r = rng.random()
        nb = rng.random() < 0.3
        if r < 0.55:
            self.put(v, nb)
        else:
            if v.is_rec and any(p[0] == "put" for p in self.pending.values()):
                self.wait()
            self.get(v, nb)

    # ------------------------------------------------------------ end
    def close_and_check(self):
        self.wait()
        assert self.N.close(self.ncid) == 0
        raw = open(self.path, "rb").read()
        h = cdfparse.parse_cdf(raw)
        assert h["numrecs"] == self.numrecs, (h["numrecs"], self.numrecs)
        byname = {x["name"]: x for x in h["vars"]}
        for v in self.vars:
            hv = byname[v.name]
            if v.is_rec:
                for r, (b, k) in v.recs.items():
                    off = hv["begin"] + r * h["recsize"]
                    seg = raw[off:off + v.per * v.xs]          # the last record may end early: an appending
                    seg += b"\0" * (v.per * v.xs - len(seg))     # put writes only up to its own last byte
                    fb = np.frombuffer(seg, np.uint8).reshape(-1, v.xs)
                    assert (fb[k] == b.reshape(-1, v.xs)[k]).all(), ("file bytes", v.name, r)
            else:
                fb = np.frombuffer(raw[hv["begin"]:hv["begin"] + v.per * v.xs], np.uint8)
                assert fb.tobytes() == v.fixed.tobytes(), ("file bytes", v.name)
        return self.counts


def run(path, seed, conv, steps=150, log_path=None, **kw):
    f = FileFuzz(path, seed, conv, **kw)
    try:
        f.create()
        f.log.append("vars " + "; ".join(f"{v.name} x{v.xtype} {v.shape}" for v in f.vars))
        for _ in range(steps):
            f.step()
        counts = f.close_and_check()
    except BaseException:
        if log_path:
            with open(log_path, "w") as fh:
                fh.write("\n".join(f.log) + "\n")
        raise
    os.unlink(path)
    return counts
