"""Repeat seeds of the file-layer fuzz (tests/file_fuzz.py) in one process
until one fails or the count runs out; the failing run's operation log goes
to gpurun_out/fuzz_repeat_<seed>_<fmt>.log.
    python tools/fuzz_repeat.py <seed:fmt,seed:fmt,...> <reps> [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests import file_fuzz  # noqa: E402
from tests.converters import OracleConv  # noqa: E402

if sys.argv[1].startswith("range"):                 # rangeA-B:fmt1/fmt2 -> seeds A..B-1 x formats
    a, b = sys.argv[1][5:].split(":")[0].split("-")
    fmts = [int(x) for x in sys.argv[1].split(":")[1].split("/")]
    cases = [(sd, fm) for sd in range(int(a), int(b)) for fm in fmts]
else:
    cases = [tuple(int(x) for x in c.split(":")) for c in sys.argv[1].split(",")]
nfail = 0
reps = int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 150
os.makedirs("gpurun_out", exist_ok=True)
conv = OracleConv()
t0 = time.time()
for k in range(reps):
    for seed, fmt in cases:
        path = f"/dev/shm/pncx_fuzz_rep_{os.getpid()}.nc"
        try:
            file_fuzz.run(path, seed, conv, steps=steps, fmt=fmt, torch=torch,
                          log_path=f"gpurun_out/fuzz_repeat_{seed}_{fmt}_{k}.log")
        except AssertionError as e:
            print(f"rep {k} seed {seed} fmt {fmt}: FAILED {e}", flush=True)
            if os.path.exists(path):
                os.unlink(path)
            nfail += 1
            if nfail >= 6:
                sys.exit(1)
    print(f"rep {k}: ok ({time.time() - t0:.1f} s)", flush=True)
print("all ok" if nfail == 0 else f"{nfail} failures")
sys.exit(1 if nfail else 0)
