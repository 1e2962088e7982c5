"""Run bench.py's C1 workload alone (the repeated-range legs, the
first_touch leg and the reference sequences) and print it as one JSON line.

    python tools/c1_bench.py [--first-only] [--nrec N]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--first-only", action="store_true")
ap.add_argument("--nrec", type=int, default=32)
a = ap.parse_args()
out = bench.c1_first_touch(nrec=a.nrec) if a.first_only else bench.c1_workload()
print(json.dumps(out), flush=True)
