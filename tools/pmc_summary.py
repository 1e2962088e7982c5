"""Summarise rocprofv3 output into profiles/ (kernel stats + HBM traffic).

    python tools/pmc_summary.py <prof_dir> <round_tag> [out_dir]

Reads <prof_dir>/trace/*_kernel_stats.csv and the FETCH_SIZE / WRITE_SIZE
counter_collection CSVs of tools/gpu_profile.sh (one counter per pass, one
pass per bench workload: <prof_dir>/pmc_fetch_<w>/, pmc_write_<w>/).  HBM
bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: rocprofv3 reports
both in KiB, and on gfx950 FETCH_SIZE counts exactly half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md §HBM), hence the factor 2.  A
step that launches several product kernels (C4 ERANGE: the PutOp batch and
the swap batch) sums their per-launch counters.  Writes
profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc.csv and updates
profiles/pmc_traffic.json (bytes per element per step, read by bench.py).
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bench workload -> (bench metric key, product kernel name patterns of one step,
# algorithmic bytes per element, elements per step at bench.py's default sizes:
# C2 32 GiB of NC_DOUBLE, C3 2^31 NC_INT, C4 256 x 2^20)
WORKLOADS = {
    "c2": ("swap8", [r"k_tile<pncx::SwapOp<8>"], 16, 1 << 32),
    "c3": ("get_int_double", [r"k_tile<pncx::GetOp<4, 9>"], 12, 1 << 31),
    "c4": ("batch_c4", [r"k_batch_swapmix"], 6, 1 << 28),
    "c4_erange": ("batch_c4_erange", [r"k_batch<pncx::PutOp<3, 8, false>", r"k_batch_swapmix"], 7, 1 << 28),
}


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def counter(prof, ctr, w, pats):
    """Mean per-launch value of one counter, summed over the step's kernels;
    None when a kernel of the step is missing from the pass."""
    vals = {p: [] for p in pats}
    sub = "pmc_fetch_" if ctr == "FETCH_SIZE" else "pmc_write_"
    for path in glob.glob(os.path.join(prof, sub + w, "**", "*_counter_collection.csv"), recursive=True):
        for r in rows(path):
            if r["Counter_Name"] != ctr:
                continue
            for p in pats:
                if re.search(re.escape(p), r["Kernel_Name"]):
                    vals[p].append(float(r["Counter_Value"]))
    if any(not v for v in vals.values()):
        return None
    return sum(sum(v) / len(v) for v in vals.values())


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    out_dir = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    for p in glob.glob(os.path.join(prof, "trace", "**", "*_kernel_stats.csv"), recursive=True):
        shutil.copy(p, os.path.join(out_dir, f"{tag}_{os.path.basename(p)}"))
    pmc_rows, kernels = [], {}
    for w, (key, pats, bpe, elems) in WORKLOADS.items():
        f, wr = counter(prof, "FETCH_SIZE", w, pats), counter(prof, "WRITE_SIZE", w, pats)
        if f is None or wr is None:
            continue
        hbm = (2 * f + wr) * 1024.0
        kernels[key] = {"workload": w, "kernels": pats, "fetch_kib": f, "write_kib": wr,
                        "hbm_bytes_per_launch": hbm, "elements_per_launch": elems,
                        "bytes_per_elem": hbm / elems, "algorithmic_bytes_per_elem": bpe,
                        "traffic_over_algorithmic": hbm / (elems * bpe)}
        pmc_rows.append([key, " + ".join(pats), f, wr, hbm, elems, hbm / elems, bpe])
    with open(os.path.join(out_dir, f"{tag}_pmc.csv"), "w", newline="") as fo:
        cw = csv.writer(fo)
        cw.writerow(["workload", "kernels", "FETCH_SIZE_KiB", "WRITE_SIZE_KiB", "hbm_bytes_corrected",
                     "elements", "bytes_per_elem", "algorithmic_bytes_per_elem"])
        cw.writerows(pmc_rows)
    p = os.path.join(out_dir, "pmc_traffic.json")
    old = json.load(open(p)) if os.path.exists(p) else {"kernels": {}}
    old["kernels"].update(kernels)
    old["_comment"] = ("HBM bytes per element from rocprofv3 PMC passes (FETCH_SIZE doubled for gfx950, "
                       "WRITE_SIZE as is; both KiB; summed over a step's product kernels); "
                       "written by tools/pmc_summary.py")
    old["round"] = tag
    old["source"] = f"profiles/{tag}_pmc.csv"
    json.dump(old, open(p, "w"), indent=1)
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main()
