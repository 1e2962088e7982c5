import os, sys, ctypes, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from pnetcdf_amd import pncx, nctypes as T, ncfile as N
n = 32 << 20
a = np.random.default_rng(3).standard_normal(n)
t = torch.from_numpy(a).cuda()
exp = a.astype(">f4").view(np.uint8)
# direct device conversion
x = torch.zeros(n * 4, dtype=torch.uint8, device="cuda")
st = torch.zeros(1, dtype=torch.int32, device="cuda")
fb = np.frombuffer(T.fill_bytes(T.NC_FLOAT) + b"\0" * 8, np.uint8).copy()
for k in range(3):
    rc = pncx.lib().pncx_dev_putn(5, T.NC_FLOAT, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(t.data_ptr()), n, T.ITYPE_DOUBLE, ctypes.c_void_p(fb.ctypes.data), ctypes.c_void_p(st.data_ptr()), None)
    torch.cuda.synchronize()
    got = x.cpu().numpy()
    bad = np.nonzero(got != exp)[0]
    print("dev_putn rc", rc, "status", int(st.item()), "bad bytes", bad.size, bad[:5] // 4 if bad.size else "")
# file path
p = "/tmp/big.nc"
err, ncid = N.create(p, N.NC_64BIT_DATA)
N.def_dim(ncid, "x", n); N.def_var(ncid, "a", T.NC_DOUBLE, [0]); N.def_var(ncid, "b", T.NC_FLOAT, [0])
N.enddef(ncid)
print("put_var_dev", N.put_var_dev(ncid, 1, t))
N.close(ncid)
raw = np.fromfile(p, np.uint8)
from tests import cdfparse
h = cdfparse.parse_cdf(raw[:4096].tobytes())
b0 = h["vars"][1]["begin"]
fileb = raw[b0:b0 + 4 * n]
bad = np.nonzero(fileb != exp)[0]
print("file bad bytes", bad.size, (bad[:8] // 4) if bad.size else "")
if bad.size:
    i = bad[0] // 4
    print("elem", i, "file", fileb[4*i:4*i+4], "exp", exp[4*i:4*i+4], "val", a[i])
    blk = sorted(set((bad // 4 // 1024).tolist()))
    print("bad tiles", len(blk), blk[:20])
