"""Per-kernel HBM bytes of the pack kernels from the FETCH_SIZE / WRITE_SIZE
passes of tools/gpu_flex_pmc.sh: mean per dispatch of (2 * FETCH_SIZE +
WRITE_SIZE) KiB (the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md
§HBM), per kernel name.  flex_bench's workloads each launch one kernel
(the contiguous control and the 2-D/3-D transposes included), so the rows
read against the algorithmic bytes n * 16 of the workload that ran it.

    python tools/flex_pmc_summary.py <dir>
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def per_kernel(d, ctr):
    vals = defaultdict(list)
    for p in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == ctr and ("pncx" in r["Kernel_Name"] or "k_" in r["Kernel_Name"]):
                name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
                vals[name].append(float(r["Counter_Value"]))
    return vals


def main(d):
    f, w = per_kernel(os.path.join(d, "fetch"), "FETCH_SIZE"), per_kernel(os.path.join(d, "write"), "WRITE_SIZE")
    print("kernel  dispatches  hbm_bytes_per_dispatch (2*FETCH+WRITE, KiB->B)")
    for k in sorted(set(f) & set(w)):
        fk, wk = sum(f[k]) / len(f[k]), sum(w[k]) / len(w[k])
        print(f"{k}  {len(f[k])}  {(2 * fk + wk) * 1024:.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
