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
    ap.add_argument("--last", type=float, default=0.5, help="trailing fraction of the trace for the idle-gap count")
    ap.add_argument("--step-kernel", default="sgd_flat",
                    help="kernel that ends each training step (per-step table over the trailing steps)")
    ap.add_argument("--last-steps", type=int, default=3, help="steady-state steps for the per-step table (0 = off)")
    ap.add_argument("--around", default="", help="print the kernel timeline (queue / stream ids) around the last "
                                                 "call of this kernel")
    ap.add_argument("--around-n", type=int, default=14)
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
    gaps(a.dir, a.last)
    if a.last_steps:
        per_step(a.dir, a.step_kernel, a.last_steps, a.top)
    if a.around:
        around(a.dir, a.around, a.around_n)


def around(d, name, n):
    """Kernel timeline (start offset, duration, idle before, queue / stream id) of the n kernels
    before and after the second-to-last call of ``name``: which stream a GPU idle gap waited on."""
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Queue_Id", "?"), r.get("Stream_Id", "?")))
    rows.sort()
    hits = [i for i, r in enumerate(rows) if name in r[2]]
    if len(hits) < 2:
        print(f"around: fewer than 2 '{name}' kernels")
        return
    c = hits[-2]
    t0 = rows[c][0]
    print(f"timeline around '{name}' (us from its start; idle = gap after the latest end so far)")
    last_end = None
    for r in rows[max(0, c - n): c + n + 1]:
        idle = "" if last_end is None else f"{max(0, r[0] - last_end) / 1e3:7.1f}"
        print(f"  {(r[0] - t0) / 1e3:9.1f} dur {(r[1] - r[0]) / 1e3:7.1f} idle {idle:>7} q {r[3]:>3} s {r[4]:>3}  {r[2][:90]}")
        last_end = r[1] if last_end is None else max(last_end, r[1])


def per_step(d, step_kernel, nsteps, top):
    """Per-kernel device time per step over the last ``nsteps`` complete steps (delimited by the
    step-ending kernel), so first-step autotuning and warm-up do not skew the attribution."""
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if step_kernel in r[2]]
    if len(ends) < nsteps + 1:
        print(f"per-step table: only {len(ends)} '{step_kernel}' kernels in the trace")
        return
    win = rows[ends[-nsteps - 1] + 1: ends[-1] + 1]
    agg = {}
    for s_, e_, n in win:
        k = _short(n) if "igemm" not in n else n.split("(")[0].replace("void ", "")
        t, c = agg.get(k, (0, 0))
        agg[k] = (t + e_ - s_, c + 1)
    span = (win[-1][1] - win[0][0]) / nsteps
    tot = sum(t for t, _ in agg.values()) / nsteps
    print(f"per step over the last {nsteps} steps: span {span / 1e3:.1f} us, kernel time {tot / 1e3:.1f} us, "
          f"{len(win) / nsteps:.0f} kernels")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"  {t / nsteps / 1e3:9.1f} us/step {100 * t / nsteps / tot:5.1f}%  calls/step={c / nsteps:6.1f}  {k[:100]}")


def gaps(d, last):
    """GPU idle time between kernels (union of kernel intervals over all queues) in the window of the
    last ``last`` kernels-per-step... approximated as the trailing 50 % of the trace (timed steps)."""
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return
    iv = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                s, e = r.get("Start_Timestamp"), r.get("End_Timestamp")
                if s and e:
                    iv.append((int(s), int(e), r.get("Kernel_Name", "?")))
    if not iv:
        return
    iv.sort()
    iv = iv[int(len(iv) * (1 - last)):]
    busy, cur_s, cur_e, n_gap, small = 0, iv[0][0], iv[0][1], 0, 0
    cur_name, by_pair = iv[0][2], {}
    for s, e, name in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            n_gap += 1
            if s - cur_e < 5000:
                small += s - cur_e
            key = (_short(cur_name), _short(name))
            t, c = by_pair.get(key, (0, 0))
            by_pair[key] = (t + s - cur_e, c + 1)
            cur_s, cur_e, cur_name = s, e, name
        elif e > cur_e:
            cur_e, cur_name = e, name
    busy += cur_e - cur_s
    span = max(x[1] for x in iv) - iv[0][0]
    print(f"trailing {100 * last:.0f}% of the trace: {len(iv)} kernels, span {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms, "
          f"idle {(span - busy) / 1e6:.2f} ms in {n_gap} gaps ({small / 1e6:.2f} ms in gaps < 5 us)")
    print("largest idle totals by (kernel that ended last -> next kernel):")
    for (a, b), (t, c) in sorted(by_pair.items(), key=lambda kv: -kv[1][0])[:15]:
        print(f"  {t / 1e6:7.3f} ms  n={c:4d} avg={t / c / 1e3:7.1f} us  {a} -> {b}")


def _short(name):
    n = name.split("(")[0].replace("void ", "")
    return n[:60]


if __name__ == "__main__":
    main()
