"""Summarise tools/gpu_pmc_pairs.sh output: per conversion kernel, the SQ
instruction / cycle counters, HBM traffic and duration, averaged over the
dispatches of the kernel in each pass.

    python tools/pmc_pairs_summary.py gpurun_out/pmc_<tag> > profiles/<tag>_pmc_pairs.txt

Derived columns (units per MI355X_MICROARCH.md: SQ_*_CYCLES and
SQ_ACTIVE_INST_* count quad-cycles; FETCH_SIZE/WRITE_SIZE are KiB and
FETCH_SIZE counts half the bytes of a wide streaming read on gfx950):
  valu/wave     SQ_INSTS_VALU / SQ_WAVES
  vmem/wave     (SQ_INSTS_VMEM_RD + SQ_INSTS_VMEM_WR) / SQ_WAVES
  valu_busy     SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES / CUs per SQ ... reported
                as SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (the share of wave
                lifetime spent issuing VALU)
  wait          SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier)
  traffic       (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes
"""
import collections
import csv
import glob
import os
import re
import sys


def load(d, sub):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for p in glob.glob(os.path.join(d, sub, "*_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if "pncx::" not in k or "k_flags" in k:
                continue
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for p in glob.glob(os.path.join(d, sub, "*_kernel_trace.csv")):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if "pncx::" not in k:
                continue
            durs[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out, durs


def short(k):
    m = re.search(r"(k_\w+)<pncx::(\w+)<([^>]*)>", k)
    return f"{m.group(1)}<{m.group(2)}<{m.group(3)}>>" if m else k[:60]


def main():
    d = sys.argv[1]
    cnt = collections.defaultdict(dict)
    for sub in ("sq", "sq2", "fetch", "write"):
        c, _ = load(d, sub)
        for k, v in c.items():
            for name, vals in v.items():
                cnt[k][name] = sum(vals) / len(vals)
    _, durs = load(d, "sq")
    hdr = ["kernel", "waves", "valu/wave", "vmem/wave", "salu/wave", "lds/wave", "valu_of_wave_cyc",
           "wait_of_wave_cyc", "inst_wait_of_wave_cyc", "traffic_GB"]
    print("  ".join(hdr))
    for k, c in cnt.items():
        w = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        row = [short(k), f"{w:.0f}", f"{c.get('SQ_INSTS_VALU', 0) / w:.1f}",
               f"{(c.get('SQ_INSTS_VMEM_RD', 0) + c.get('SQ_INSTS_VMEM_WR', 0)) / w:.1f}",
               f"{c.get('SQ_INSTS_SALU', 0) / w:.1f}", f"{c.get('SQ_INSTS_LDS', 0) / w:.1f}",
               f"{c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}", f"{c.get('SQ_WAIT_ANY', 0) / wc:.3f}",
               f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}",
               f"{(2 * c.get('FETCH_SIZE', 0) + c.get('WRITE_SIZE', 0)) * 1024 / 1e9:.3f}"]
        print("  ".join(row))
    print()
    print("raw means per dispatch:")
    for k, c in cnt.items():
        print(short(k), {n: round(v) for n, v in sorted(c.items())})


if __name__ == "__main__":
    main()
