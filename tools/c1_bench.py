"""Run bench.py's C1 workload alone (the repeated-range legs, the
first_touch leg and the reference sequences) and print it as one JSON line.

    python tools/c1_bench.py [--first-only] [--nrec N] [--reps R] [--summary]

--summary prints bench.c1_first_summary of the first-touch legs (the form
the bench line carries) instead of the whole result.
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
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--summary", action="store_true")
a = ap.parse_args()
out = bench.c1_first_touch(nrec=a.nrec, reps=a.reps) if a.first_only else bench.c1_workload()
if a.summary:
    out = bench.c1_first_summary(out if a.first_only else out["first_touch"])
print(json.dumps(out), flush=True)
