"""Quick first-contact probe of libpncx on a GPU box (not a test)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pnetcdf_amd import nctypes as T, pncx  # noqa: E402
from oracle import oracle as O  # noqa: E402

print("torch", torch.__version__, "hip", torch.version.hip, "cuda avail", torch.cuda.is_available())
print("lib", pncx.version(), "devices", pncx.device_count())

# 1. device in-place swap
a = np.random.default_rng(1).integers(0, 2**63, 1 << 20, dtype=np.uint64)
t = torch.from_numpy(a.copy()).cuda()
pncx.dev_in_swapn(t, a.size, 8)
torch.cuda.synchronize()
ok = np.array_equal(t.cpu().numpy(), a.byteswap())
print("dev_in_swapn 8:", ok)

# 2. host swap
for es in (2, 4, 8, 3):
    b = np.random.default_rng(es).integers(0, 255, 4096 * es + es * 7, dtype=np.uint8)
    ref = b.copy()
    O.in_swapn(ref, es)
    got = b.copy()
    pncx.in_swapn(got, got.size // es, es)
    print("host in_swapn", es, np.array_equal(ref, got))

# 3. a few conversions vs oracle
rng = np.random.default_rng(7)
bad = 0
for xt in T.NUMERIC_XTYPES:
    for it in T.NUMERIC_ITYPES:
        n = 1000 + int(rng.integers(0, 50))
        raw = rng.integers(0, 256, n * 8, dtype=np.uint8)
        ib = np.frombuffer(raw.tobytes(), dtype=T.ITYPE_NP[it])[:n].copy()
        xb_ref, st_ref = O.putn(5, xt, ib, it, fill=T.fill_bytes(xt))
        xb = np.zeros(n * T.xlen(xt), np.uint8)
        st = pncx.putn(5, xt, xb, ib, n, it, T.fill_bytes(xt))
        if xb.tobytes() != xb_ref or st != st_ref:
            bad += 1
            print("PUT mismatch", T.XNAME[xt], T.INAME[it], st, st_ref)
        xraw = rng.integers(0, 256, n * T.xlen(xt), dtype=np.uint8)
        ir, st_ref = O.getn(5, xt, xraw.tobytes(), it)
        ig = np.zeros(n, T.ITYPE_NP[it])
        st = pncx.getn(5, xt, xraw, ig, n, it)
        if ig.tobytes() != ir.tobytes() or st != st_ref:
            bad += 1
            d = np.nonzero(ig.view(np.uint8).reshape(n, -1).any(1) != ir.view(np.uint8).reshape(n, -1).any(1))
            print("GET mismatch", T.XNAME[xt], T.INAME[it], st, st_ref,
                  [(i, ig[i], ir[i]) for i in np.nonzero(ig.tobytes() != ir.tobytes())[0][:3]] if False else "")
print("conversion mismatches:", bad)

# 4. timing: 8 GiB in-place 8-byte swap
n = (8 << 30) // 8
big = torch.empty(n, dtype=torch.int64, device="cuda")
big.random_()
torch.cuda.synchronize()
for nt in (0, 1):
    import os
    os.environ["PNCX_NONTEMPORAL"] = str(nt)
    for _ in range(2):
        pncx.dev_in_swapn(big, n, 8)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    reps = 10
    for _ in range(reps):
        pncx.dev_in_swapn(big, n, 8)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print(f"8GiB in-place swap nt={nt}: {ms:.3f} ms  {2*8*n/ms/1e6:.1f} GB/s")
