"""Workload for the host-side ASan build (tools/asan/run.sh): every CDF
fixture the reference's tests hold, the no-conversion data paths, error
paths that end in the no-device stub, and a mutation fuzz of the header
decoder (open + validate of corrupted headers must never touch memory it
does not own)."""
import os
import random
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pnetcdf_amd import nctypes as T          # noqa: E402
from pnetcdf_amd import ncfile as N           # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def walk(ncid):
    err, nd, nv, ng, ul = N.inq(ncid)
    for d in range(nd):
        N.inq_dim(ncid, d)
    for a in range(ng):
        e, name = N.inq_attname(ncid, N.NC_GLOBAL, a)
        e, xt, n = N.inq_att(ncid, N.NC_GLOBAL, name)
        if xt == T.NC_CHAR:
            N.get_att(ncid, N.NC_GLOBAL, name)
    for v in range(nv):
        e, name, xt, dims, na = N.inq_var(ncid, v)
        N.inq_varoffset(ncid, v)
        if xt in (T.NC_CHAR, T.NC_BYTE) and len(dims) <= 3:
            shape = [N.inq_dim(ncid, d)[2] for d in dims]
            n = int(np.prod(shape)) if shape else 1
            if n <= 1 << 16:
                out = np.zeros(max(n, 1), "S1" if xt == T.NC_CHAR else np.int8)
                N.get_var(ncid, v, out)


def fixtures():
    files = [os.path.join(GOLD, "cdf", f) for f in sorted(os.listdir(os.path.join(GOLD, "cdf")))]
    files.append(os.path.join(GOLD, "tst_file.nc"))
    for f in files:
        err, ncid = N.open(f)
        if err == 0:
            walk(ncid)
            N.close(ncid)
        N.validate(f)
    print("fixtures ok", len(files))


def data_paths(td):
    p = os.path.join(td, "d.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    N.def_dim(ncid, "t", N.NC_UNLIMITED)
    N.def_dim(ncid, "y", 33)
    N.def_dim(ncid, "x", 1000)
    N.def_var(ncid, "c", T.NC_CHAR, [1, 2])
    N.def_var(ncid, "r", T.NC_BYTE, [0, 2])
    N.def_var(ncid, "i", T.NC_INT, [1, 2])
    N.put_att_text(ncid, N.NC_GLOBAL, "title", "asan")
    assert N.enddef(ncid) == 0
    a = np.frombuffer(bytes(range(256)) * 129, "S1")[:33000].copy()
    assert N.put_var(ncid, 0, a) == 0
    assert N.put_var(ncid, 0, a[:99].copy(), [1, 2], [3, 33], [5, 7]) == 0
    b = np.arange(4000, dtype=np.int8)
    reqs = [N.iput_var(ncid, 1, b[k * 1000:(k + 1) * 1000].copy(), [k, 0], [1, 1000])[1] for k in (3, 0, 2, 1)]
    N.wait_all(ncid, reqs)
    out = np.zeros(4000, np.int8)
    N.get_var(ncid, 1, out, [0, 0], [4, 1000])
    assert N.put_var(ncid, 2, np.arange(33000, dtype=np.int32)) == N.PNCX_EDEVICE   # no device: loud
    N.iput_var(ncid, 2, np.arange(1000, dtype=np.int32), [0, 0], [1, 1000])
    N.wait_all(ncid)
    for bad in ([40, 0], [-1, 0], [0, 999]):
        N.put_var(ncid, 0, a[:10].copy(), bad, [1, 10])
    # varn and buffered puts (copy paths)
    N.put_varn(ncid, 0, [[0, 0], [5, 5], [7, 0]], [[1, 10], None, [2, 3]], a[:17].copy())
    o17 = np.zeros(17, "S1")
    N.get_varn(ncid, 0, [[0, 0], [5, 5], [7, 0]], [[1, 10], None, [2, 3]], o17)
    N.buffer_attach(ncid, 4096)
    rq = [N.bput_var(ncid, 1, b[:100].copy(), [k, 0], [1, 100])[1] for k in range(5)]
    N.bput_var(ncid, 1, b[:4000].copy(), [0, 0], [4, 1000])           # NC_EINSUFFBUF
    N.wait_all(ncid, rq[::-1])
    N.buffer_detach(ncid)
    assert N.redef(ncid) == 0
    for k in range(30):
        N.put_att_text(ncid, N.NC_GLOBAL, f"a{k}", "x" * k)
    N.def_var(ncid, "later", T.NC_CHAR, [2])
    N.rename_var(ncid, 0, "cc")
    N.del_att(ncid, N.NC_GLOBAL, "a3")
    assert N._enddef(ncid, 100, 1024, 16, 8) == 0
    o = np.zeros(33000, "S1")
    N.get_var(ncid, 0, o)
    N.iput_var(ncid, 0, a[:10].copy(), [0, 0], [1, 10])
    N.close(ncid)                                   # pending request -> NC_EPENDING path
    err, ncid = N.open(p)
    walk(ncid)
    N.close(ncid)
    print("data paths ok")


def fuzz(td, rounds):
    rng = random.Random(1234)
    seeds = [open(os.path.join(GOLD, "tst_file.nc"), "rb").read()]
    for v in (1, 2, 5):
        seeds.append(open(os.path.join(GOLD, "cdf", f"test_cdf.nc{v}"), "rb").read())
    # a richer seed: many dims/atts/vars in CDF-5
    p = os.path.join(td, "seed.nc")
    err, ncid = N.create(p, N.NC_64BIT_DATA)
    for d in range(6):
        N.def_dim(ncid, f"d{d}", 0 if d == 0 else d + 2)
    for k in range(5):
        N.put_att_text(ncid, N.NC_GLOBAL, f"g{k}", "v" * (k + 1))
    for k in range(8):
        N.def_var(ncid, f"v{k}", T.NC_CHAR if k % 2 else T.NC_BYTE, [0, 1 + k % 5] if k % 3 else [2, 3])
        N.put_att_text(ncid, k, "units", "m" * k)
    N.enddef(ncid)
    N.close(ncid)
    seeds.append(open(p, "rb").read())
    path = os.path.join(td, "f.nc")
    opened = 0
    for it in range(rounds):
        s = bytearray(rng.choice(seeds))
        hdr = min(len(s), 600)
        for _ in range(rng.randint(1, 6)):
            kind = rng.random()
            pos = rng.randrange(4, max(5, hdr))
            if kind < 0.5 and pos < len(s):
                s[pos] = rng.randrange(256)
            elif kind < 0.7 and pos + 4 <= len(s):          # a length/count field -> huge or zero
                s[pos:pos + 4] = rng.choice([b"\xff\xff\xff\xff", b"\x7f\xff\xff\xff", b"\x00\x00\x00\x00",
                                            b"\x00\x00\x01\x00"])
            elif kind < 0.85:
                del s[pos:]                                   # truncation
            else:
                s[pos:pos] = bytes(rng.randrange(256) for _ in range(rng.randint(1, 9)))
        with open(path, "wb") as f:
            f.write(s)
        err, ncid = N.open(path)
        if err == 0:
            opened += 1
            walk(ncid)
            N.close(ncid)
        N.validate(path)
    print("fuzz ok", rounds, "mutants,", opened, "opened")


if __name__ == "__main__":
    with tempfile.TemporaryDirectory() as td:
        fixtures()
        data_paths(td)
        fuzz(td, int(os.environ.get("FUZZ_ROUNDS", "4000")))
