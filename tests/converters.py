"""Uniform converter adapters for the reference-test restatements:
the CPU oracle (checker) and the HIP library (host and device entry points)."""
import numpy as np

from pnetcdf_amd import nctypes as T


class OracleConv:
    name = "oracle"

    def __init__(self):
        from oracle import oracle as O
        self.O = O

    def putn(self, cdf, xtype, ibuf, itype, fill, xinit=None):
        return self.O.putn(cdf, xtype, np.ascontiguousarray(ibuf, T.ITYPE_NP[itype]), itype,
                           fill=fill, xinit=xinit)

    def getn(self, cdf, xtype, xbytes, itype):
        return self.O.getn(cdf, xtype, xbytes, itype)


class HipHostConv:
    """include/pncx.h host-buffer entry points (staged through HBM)."""
    name = "hip-host"

    def __init__(self):
        from pnetcdf_amd import pncx as P
        self.P = P

    def putn(self, cdf, xtype, ibuf, itype, fill, xinit=None):
        ibuf = np.ascontiguousarray(ibuf, T.ITYPE_NP[itype])
        n = ibuf.size
        if xinit is None:
            xb = np.zeros(n * T.xlen(xtype), np.uint8)
        else:
            xb = np.frombuffer(bytes(xinit), np.uint8).copy()
        st = self.P.putn(cdf, xtype, xb, ibuf, n, itype, fill)
        return xb.tobytes(), st

    def getn(self, cdf, xtype, xbytes, itype):
        xb = np.frombuffer(bytes(xbytes), np.uint8).copy()
        n = xb.size // T.xlen(xtype)
        out = np.zeros(n, T.ITYPE_NP[itype])
        st = self.P.getn(cdf, xtype, xb, out, n, itype)
        return out, st


class HipDevConv:
    """include/pncx.h device entry points on torch HBM tensors."""
    name = "hip-dev"

    def __init__(self):
        import torch
        from pnetcdf_amd import pncx as P
        self.P, self.torch = P, torch

    def _dev(self, arr):
        return self.torch.from_numpy(np.frombuffer(arr.tobytes(), np.uint8).copy()).cuda()

    def putn(self, cdf, xtype, ibuf, itype, fill, xinit=None):
        torch = self.torch
        ibuf = np.ascontiguousarray(ibuf, T.ITYPE_NP[itype])
        n = ibuf.size
        di = self._dev(ibuf) if n else torch.zeros(16, dtype=torch.uint8, device="cuda")
        if xinit is None:
            dx = torch.zeros(max(n * T.xlen(xtype), 16), dtype=torch.uint8, device="cuda")
        else:
            dx = self._dev(np.frombuffer(bytes(xinit), np.uint8))
        ds = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.P.dev_putn(cdf, xtype, dx, di, n, itype, fill, ds)
        torch.cuda.synchronize()
        return dx.cpu().numpy()[: n * T.xlen(xtype)].tobytes(), int(ds.item())

    def getn(self, cdf, xtype, xbytes, itype):
        torch = self.torch
        xs = T.xlen(xtype)
        n = len(xbytes) // xs
        dx = self._dev(np.frombuffer(bytes(xbytes), np.uint8)) if n else torch.zeros(16, dtype=torch.uint8, device="cuda")
        di = torch.zeros(max(n * T.ilen(itype), 16), dtype=torch.uint8, device="cuda")
        ds = torch.zeros(1, dtype=torch.int32, device="cuda")
        self.P.dev_getn(cdf, xtype, dx, di, n, itype, ds)
        torch.cuda.synchronize()
        out = np.frombuffer(di.cpu().numpy()[: n * T.ilen(itype)].tobytes(), T.ITYPE_NP[itype]).copy()
        return out, int(ds.item())
