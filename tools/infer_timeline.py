"""Per-image view of a rocprofv3 kernel trace of the batch-1 hipGraph inference loop
(tools/prof_infer.py): kernels and GPU span per image (median over the last 100 images) and the kernel
timeline of one steady-state image.  Usage: python tools/infer_timeline.py <rocprof dir>"""
import csv
import glob
import os
import statistics
import sys


def main(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    groups, cur = [], [ts[0]]
    for b in ts[1:]:
        if b[0] - max(x[1] for x in cur[-8:]) > 20000:   # > 20 us idle: the next image
            groups.append(cur)
            cur = []
        cur.append(b)
    groups.append(cur)
    groups = [g for g in groups if len(g) > 10][-100:]
    span = [(max(e for _, e, _ in g) - g[0][0]) / 1e3 for g in groups]
    nk = [len(g) for g in groups]
    print(f"per inference: kernels {statistics.median(nk)}, GPU span {statistics.median(span):.1f} us")
    g = groups[len(groups) // 2]
    t0, last_end = g[0][0], g[0][0]
    print("one image's kernels: start / dur / gap-after-latest-end (us)")
    for s, e, n in g:
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {(s - last_end) / 1e3:7.1f}  {n[:110]}")
        last_end = max(last_end, e)


if __name__ == "__main__":
    main(sys.argv[1])
