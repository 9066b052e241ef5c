"""End-of-backward tail of a training step (rocprofv3 --kernel-trace CSV): when does the compute
stream (the SGD kernel's stream) run out of work, when does the side stream finish its queued
WGRADs, and which kernels fill the gap before the optimizer step.

Usage: python tools/tail_report.py <rocprof dir> [--steps 3] [--last 14]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--last", type=int, default=14)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    sgd = [i for i, r in enumerate(rows) if "sgd_flat" in r["Kernel_Name"]]
    for k in range(max(1, len(sgd) - a.steps), len(sgd)):
        step = rows[sgd[k - 1] + 1:sgd[k] + 1]
        s_sgd = int(step[-1]["Start_Timestamp"])
        t0 = int(step[0]["Start_Timestamp"])
        main = step[-1]["Stream_Id"]
        comp = [r for r in step[:-1] if r["Stream_Id"] == main]
        side = [r for r in step[:-1] if r["Stream_Id"] != main]
        c_end = max(int(r["End_Timestamp"]) for r in comp)
        s_end = max(int(r["End_Timestamp"]) for r in side) if side else c_end
        busy_c = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in comp)
        busy_s = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in side)
        print(f"step {k}: span {(s_sgd - t0) / 1e3:8.1f} us to the SGD kernel; compute stream busy {busy_c / 1e3:8.1f} us, "
              f"side streams busy {busy_s / 1e3:8.1f} us; compute stream's last kernel ends {(s_sgd - c_end) / 1e3:6.1f} us "
              f"before SGD, side streams' {(s_sgd - s_end) / 1e3:6.1f} us before (tail wait {max(0, s_end - c_end) / 1e3:.1f} us)")
        for r in step[-a.last - 1:]:
            st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            tag = "C" if r["Stream_Id"] == main else "S" + r["Stream_Id"]
            print(f"    {tag:>4} {(st - s_sgd) / 1e3:9.1f} .. {(en - s_sgd) / 1e3:9.1f} us  {r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
