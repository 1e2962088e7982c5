"""Summarise tools/gpu_scatter_pmc.sh: per mode, the mean of each counter over
the timed dispatches (the first, warm-up dispatch dropped), per element and
per launch-microsecond.  python tools/scatter_pmc_summary.py <dir>"""
import csv
import glob
import os
import sys

ELEMS = 33551134 * 8                       # tools/scatter_probe.hip's layout
d = sys.argv[1]
rows = {}
for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
    mode = os.path.basename(os.path.dirname(f)).split(".")[0]
    per = {}
    for r in csv.DictReader(open(f)):
        per.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
        per[int(r["Dispatch_Id"])]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(per)[1:]
    for k in set().union(*(per[i].keys() for i in ids)):
        if k == "_ns":
            continue
        rows.setdefault(mode, {})[k] = sum(per[i].get(k, 0) for i in ids) / len(ids)
    rows.setdefault(mode, {}).setdefault("_ns", []).extend(per[i]["_ns"] for i in ids)
order = [m for m in ["gather", "nt", "wb", "touch", "touch2", "touch2nt", "fill"] if m in rows]
keys = sorted({k for m in rows.values() for k in m if k != "_ns"})
print("counter (per element, mean over timed launches)".ljust(40) + "".join(m.rjust(12) for m in order))
print("launch us".ljust(40) + "".join(f"{sum(rows[m]['_ns']) / len(rows[m]['_ns']) / 1e3:12.1f}" for m in order))
for k in keys:
    print(k.ljust(40) + "".join(f"{rows[m].get(k, float('nan')) / ELEMS:12.4f}" for m in order))
print("derived")
for m in order:
    r = rows[m]
    wr, w64, rd = r.get("TCC_EA0_WRREQ", 0), r.get("TCC_EA0_WRREQ_64B", 0), r.get("TCC_EA0_RDREQ", 0)
    us = sum(r["_ns"]) / len(r["_ns"]) / 1e3
    print(f"  {m:7s} write requests {wr / ELEMS:.3f}/elem, of them 64B {w64 / max(wr, 1):.3f}; "
          f"write bytes ~{(64 * w64 + 32 * (wr - w64)) / ELEMS:.2f}/elem; read req {rd / ELEMS:.3f}/elem; "
          f"write stall cycles/req {r.get('TCC_EA0_WRREQ_STALL', 0) / max(wr, 1):.2f}; "
          f"DRAM credit stall {r.get('TCC_EA0_WRREQ_DRAM_CREDIT_STALL', 0) / max(wr, 1):.2f}; "
          f"TA busy {r.get('TA_BUSY', 0) / max(r.get('GRBM_GUI_ACTIVE', 1), 1):.2f} x GUI")
