"""Summarise tools/gpu_c4_pmc.sh: per mode (batch / flat2 / flat), the mean
of each counter over the timed dispatches of the conversion kernel (the
first, warm-up dispatch dropped), and what they say about ramp/drain and
DRAM placement.  python tools/c4_pmc_summary.py <dir>"""
import csv
import glob
import json
import os
import sys

MOVED = 2 * 128 * (1 << 20) * 6            # C4: 768 MiB read + 768 MiB written

d = sys.argv[1]
rows, names = {}, {}
for f in sorted(glob.glob(os.path.join(d, "*", "p_counter_collection.csv"))):
    mode = os.path.basename(os.path.dirname(f)).split(".")[0]
    per = {}
    for r in csv.DictReader(open(f)):
        kn = r["Kernel_Name"]
        if "batch" not in kn and "k_tile" not in kn:
            continue
        names[mode] = kn.split("(")[0][:60]
        i = int(r["Dispatch_Id"])
        per.setdefault(i, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        per[i]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(per)[1:]
    if not ids:
        continue
    m = rows.setdefault(mode, {"_ns": []})
    for k in set().union(*(per[i].keys() for i in ids)) - {"_ns"}:
        m.setdefault(k, []).append(sum(per[i].get(k, 0) for i in ids) / len(ids))
    m["_ns"] += [per[i]["_ns"] for i in ids]
out = {}
for mode in [x for x in ("batch", "flat2", "flat") if x in rows]:
    r = {k: (sum(v) / len(v)) for k, v in rows[mode].items()}
    us = r["_ns"] / 1e3
    gui = r.get("GRBM_GUI_ACTIVE", 0.0)
    xcd_cycles = gui / 8                    # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs
    rd, wr = r.get("TCC_EA0_RDREQ", 0.0), r.get("TCC_EA0_WRREQ", 0.0)
    t = {"kernel": names.get(mode), "launch_us_under_pmc": round(us, 1),
         "frac_of_8TBs_under_pmc": round(MOVED / (us * 1e-6) / 8e12, 4),
         "clock_GHz": round(xcd_cycles / (us * 1e3), 3),
         "waves": r.get("SQ_WAVES"),
         # SQ_WAVE_CYCLES counts quad-cycles summed over waves
         "mean_resident_waves": round(4 * r.get("SQ_WAVE_CYCLES", 0) / max(xcd_cycles, 1), 1),
         "sq_busy_share": round(r.get("SQ_BUSY_CYCLES", 0) / max(gui, 1), 3),
         "read_req_per_MiB": round(rd / (MOVED / 2 / (1 << 20)), 1),
         "write_req_per_MiB": round(wr / (MOVED / 2 / (1 << 20)), 1),
         "write_64B_share": round(r.get("TCC_EA0_WRREQ_64B", 0) / max(wr, 1), 3),
         "rd_dram_credit_stall_per_req": round(r.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL", 0) / max(rd, 1), 3),
         "wr_dram_credit_stall_per_req": round(r.get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL", 0) / max(wr, 1), 3),
         "rd_queue_level": round(r.get("TCC_EA0_RDREQ_LEVEL", 0) / max(gui, 1), 2),
         "wr_queue_level": round(r.get("TCC_EA0_WRREQ_LEVEL", 0) / max(gui, 1), 2)}
    try:
        t["events"] = json.load(open(os.path.join(d, f"{mode}.time.json")))
    except (OSError, ValueError):
        pass
    out[mode] = t
    print(json.dumps({"mode": mode, **t}))
