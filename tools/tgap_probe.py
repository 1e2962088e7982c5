"""Typemap offsets (bytes from the lowest element) of test_gpu_flex.py's
test_flex_large_table buftype (2^16 runs of 1..7 doubles, gaps 0..4), written
as uint32 for tools/tgap_probe.  Prints the probe's arguments."""
import sys

import numpy as np

rng = np.random.default_rng(5)
nb = 1 << 16
blen = rng.integers(1, 8, nb)
gaps = rng.integers(0, 5, nb)
disp = np.concatenate([[0], np.cumsum(blen + gaps)[:-1]]).astype(np.int64)
isz = 8
ext = int(disp[-1] + blen[-1] + 3) * isz
one = np.concatenate([d * isz + isz * np.arange(b) for d, b in zip(disp, blen)])
(one - one.min()).astype(np.uint32).tofile(sys.argv[1])
print(4, ext, isz)
