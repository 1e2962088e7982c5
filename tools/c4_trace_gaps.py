"""Where the synchronous C4 call's time goes outside its kernel: reads a
rocprofv3 --kernel-trace CSV of `bench.py --workload c4` (tools/
gpu_c4_trace.sh) and reports, per call, the batch kernel, the gap to the
completion block (k_batch_done), its duration, and the gap from its end to
the next call's batch kernel (host: poll, return, the next call's plan
check and launch; GPU: the idle queue's dispatch), as medians in us."""
import csv
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    ks.sort(key=lambda x: x[1])
    batch, gap1, done, gap2 = [], [], [], []
    for i in range(len(ks) - 2):
        n0, s0, e0 = ks[i]
        n1, s1, e1 = ks[i + 1]
        n2, s2, e2 = ks[i + 2]
        if "k_batch_swapmix" in n0 and "k_batch_done" in n1 and "k_batch_swapmix" in n2:
            batch.append((e0 - s0) / 1e3)
            gap1.append((s1 - e0) / 1e3)
            done.append((e1 - s1) / 1e3)
            gap2.append((s2 - e1) / 1e3)
    med = statistics.median
    if not batch:
        print("no batch/done pairs found")
        return 1
    tot = med(batch) + med(gap1) + med(done) + med(gap2)
    print(f"calls {len(batch)}: batch kernel {med(batch):.1f} us, gap to done {med(gap1):.1f}, "
          f"done block {med(done):.1f}, done end -> next batch start {med(gap2):.1f}; "
          f"per call {tot:.1f} us ({tot / med(batch):.4f} x kernel)")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
