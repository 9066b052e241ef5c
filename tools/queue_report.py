"""Which hardware queue each HIP stream's kernels ran on (rocprofv3 --kernel-trace CSV), and the
overlap between streams in the last complete training step (delimited by the SGD kernel).

Usage: python tools/queue_report.py <rocprof dir> [<rocprof dir> ...]
"""
import csv
import glob
import os
import sys
from collections import Counter


def report(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd_flat" in r["Kernel_Name"]]
    step = rows[sgd[-2] + 1:sgd[-1] + 1]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    print(f"== {d}: last step {len(step)} kernels, span {(t1 - t0) / 1e6:.2f} ms")
    by = Counter((r["Stream_Id"], r["Queue_Id"]) for r in step)
    for (s, q), n in sorted(by.items()):
        ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step if r["Stream_Id"] == s)
        print(f"  stream {s:>3} -> hw queue {q:>3}: {n:4d} kernels, {ns / 1e6:6.2f} ms of kernel time")
    # time during which kernels of >= 2 streams run at once
    ev = []
    for r in step:
        ev.append((int(r["Start_Timestamp"]), 1, r["Stream_Id"]))
        ev.append((int(r["End_Timestamp"]), -1, r["Stream_Id"]))
    ev.sort()
    act = Counter()
    last, both, busy = ev[0][0], 0, 0
    for t, k, s in ev:
        live = [x for x, c in act.items() if c > 0]
        if live:
            busy += t - last
            if len(live) >= 2:
                both += t - last
        act[s] += k
        last = t
    print(f"  GPU busy {busy / 1e6:.2f} ms; >= 2 streams concurrently {both / 1e6:.2f} ms")


if __name__ == "__main__":
    for d in sys.argv[1:]:
        report(d)
