"""Per-phase cost of a 4 MiB host-buffer swap call (pncx_in_swapn, staged
zero copy in 4 chunks), phases 1 and 2, to find what the enqueue costs.
Not product code."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pnetcdf_amd import pncx as P
n = 1 << 20
a = np.arange(n, dtype=np.uint32)
P.in_swapn(a, n, 4)
for mode in (1, 2):
    P.lib().pncx_phases(mode)
    t = []
    for _ in range(50):
        t0 = time.perf_counter()
        P.in_swapn(a, n, 4)
        t.append(time.perf_counter() - t0)
    s = P.phase_sums()
    P.lib().pncx_phases(0)
    print("mode", mode, "median call us %.1f" % (1e6 * sorted(t)[25]),
          {k: round(v[0] / 50, 2) for k, v in s.items() if v[1]}, flush=True)
