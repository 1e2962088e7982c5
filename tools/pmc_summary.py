"""Summarise rocprofv3 output into profiles/ (kernel stats + HBM traffic).

    python tools/pmc_summary.py <prof_dir> <round_tag>

Reads <prof_dir>/trace/*_kernel_stats.csv and the FETCH_SIZE / WRITE_SIZE
counter_collection CSVs (one counter per pass).  HBM bytes per launch =
(2 * FETCH_SIZE + WRITE_SIZE) * 1024: rocprofv3 reports both in KiB, and on
gfx950 FETCH_SIZE counts exactly half the bytes of a wide coalesced
streaming read (MI355X_MICROARCH.md §HBM), hence the factor 2.  Writes
profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc.csv and updates
profiles/pmc_traffic.json (bytes per element per kernel, read by bench.py).
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# product kernel name pattern -> (bench metric key, algorithmic bytes per element,
# elements per launch at bench.py's default sizes: C2 32 GiB of NC_DOUBLE,
# C3 2^31 NC_INT, C4 256 x 2^20)
KERNELS = {
    r"k_tile<pncx::SwapOp<8>": ("swap8", 16, 1 << 32),
    r"k_tile<pncx::GetOp<4, 9>": ("get_int_double", 12, 1 << 31),
    r"k_batch_swapmix": ("batch_c4", 6, 1 << 28),
}


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    prof, tag = sys.argv[1], sys.argv[2]
    out_dir = os.path.join(ROOT, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    for p in glob.glob(os.path.join(prof, "trace", "*_kernel_stats.csv")):
        shutil.copy(p, os.path.join(out_dir, f"{tag}_{os.path.basename(p)}"))
    per = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for p in glob.glob(os.path.join(prof, "pmc_*", "*_counter_collection.csv")):
            for r in rows(p):
                if r["Counter_Name"] != ctr:
                    continue
                for pat, (key, bpe, elems) in KERNELS.items():
                    if re.search(re.escape(pat), r["Kernel_Name"]):
                        per.setdefault(key, {}).setdefault(ctr, []).append(float(r["Counter_Value"]))
    pmc_rows = []
    traffic = {"_comment": "HBM bytes per element from rocprofv3 PMC passes (FETCH_SIZE doubled for "
                           "gfx950, WRITE_SIZE as is; both KiB); written by tools/pmc_summary.py",
               "round": tag, "kernels": {}}
    for key, d in per.items():
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
        w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
        bpe, elems = [(b, e) for k, b, e in KERNELS.values() if k == key][0]
        hbm = (2 * f + w) * 1024.0
        traffic["kernels"][key] = {"fetch_kib": f, "write_kib": w, "hbm_bytes_per_launch": hbm,
                                   "elements_per_launch": elems, "bytes_per_elem": hbm / elems,
                                   "algorithmic_bytes_per_elem": bpe,
                                   "traffic_over_algorithmic": hbm / (elems * bpe)}
        pmc_rows.append([key, f, w, hbm, elems, hbm / elems, bpe])
    with open(os.path.join(out_dir, f"{tag}_pmc.csv"), "w", newline="") as fo:
        wr = csv.writer(fo)
        wr.writerow(["kernel", "FETCH_SIZE_KiB", "WRITE_SIZE_KiB", "hbm_bytes_corrected", "elements",
                     "bytes_per_elem", "algorithmic_bytes_per_elem"])
        wr.writerows(pmc_rows)
    p = os.path.join(out_dir, "pmc_traffic.json")
    old = json.load(open(p)) if os.path.exists(p) else {"kernels": {}}
    old["kernels"].update(traffic["kernels"])
    old["_comment"], old["round"] = traffic["_comment"], tag
    json.dump(old, open(p, "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
