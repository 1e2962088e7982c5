"""HBM bytes per dispatch of flex_bench workloads in launch order: the pack
kernels' dispatches of one FETCH_SIZE / WRITE_SIZE pass (tools/gpu_short_ab.sh)
sorted by dispatch id and cut into groups of 1 + 10 * reps (flex_bench's
timeit: one warm launch, reps x 10 timed), labelled by the workloads that
flex_bench printed in the same order.  bytes = (2 * FETCH_SIZE + WRITE_SIZE)
KiB (the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md §HBM), over the
workload's algorithmic bytes n * 16.

    python tools/flex_pmc_seq.py <dir with fetch/ write/ fetch.log> <reps>
"""
import csv
import glob
import json
import os
import re
import sys


def seq(d, ctr):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == ctr and re.search(r"\bk_\w+", r["Kernel_Name"]):
                rows.append((int(r["Dispatch_Id"]), re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", ""),
                             float(r["Counter_Value"])))
    return sorted(rows)


def main(d, reps):
    per = 1 + 10 * reps
    wl = [json.loads(x) for x in open(os.path.join(d, "fetch.log")) if x.startswith("{")]
    f, w = seq(os.path.join(d, "fetch"), "FETCH_SIZE"), seq(os.path.join(d, "write"), "WRITE_SIZE")
    print("workload  kernel  dispatches  hbm_bytes_per_dispatch  algorithmic  ratio")
    for i, x in enumerate(wl):
        fg, wg = f[i * per:(i + 1) * per], w[i * per:(i + 1) * per]
        if len(fg) < per or len(wg) < per:
            print(f"{x['workload']}  (missing dispatches: {len(fg)} / {len(wg)})")
            continue
        b = (2 * sum(v for _, _, v in fg) / per + sum(v for _, _, v in wg) / per) * 1024
        alg = x["n"] * 16
        print(f"{x['workload']}  {fg[0][1]}  {per}  {b:.4g}  {alg:.4g}  {b / alg:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
