"""Summarise a rocprofv3 ``--stats`` run: top kernels by total time (ms), share, calls, average.

Usage: python tools/prof_summary.py <rocprof output dir> [--steps N] [--top 30]
Finds ``*kernel_stats.csv`` under the directory (rocprofv3 -d DIR --stats --kernel-trace).
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=0, help="steps profiled (prints ms/step)")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_stats.csv under {a.dir}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])))
    tot = sum(r[2] for r in rows)
    rows.sort(key=lambda r: -r[2])
    for name, calls, ns in rows[: a.top]:
        print(f"{ns / 1e6:9.2f}ms {100 * ns / tot:6.2f}% calls={calls:6d} avg={ns / calls / 1e3:9.1f}us  {name[:110]}")
    msg = f"total kernel ms {tot / 1e6:.2f}"
    if a.steps:
        msg += f" ({tot / 1e6 / a.steps:.2f} ms/step over {a.steps} steps)"
    print(msg)


if __name__ == "__main__":
    main()
