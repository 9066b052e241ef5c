"""Critical-path view of a rocprofv3 kernel trace of the training step: per stream (HIP queue) busy
time per step, the compute stream's idle gaps (what it waited for), and the forward / backward split
of the compute stream (the loss kernel divides them).

Usage: python tools/stream_report.py <rocprof dir> [--step-kernel sgd_flat] [--steps 4] [--gaps 20]
"""
import argparse
import csv
import glob
import os


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             r.get("Stream_Id", r.get("Queue_Id", "?"))))
    rows.sort()
    return rows


def short(n):
    n = n.replace("void ", "")
    return n.split("(")[0][:80]


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--step-kernel", default="sgd_flat")
    ap.add_argument("--loss-kernel", default="xent_kernel")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--gaps", type=int, default=20)
    a = ap.parse_args()
    rows = load(a.dir)
    ends = [i for i, r in enumerate(rows) if a.step_kernel in r[2]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} '{a.step_kernel}' kernels")
    comp = rows[ends[-1]][3]
    win = rows[ends[-a.steps - 1] + 1: ends[-1] + 1]
    t0, t1 = win[0][0], max(r[1] for r in win)
    span = (t1 - t0) / a.steps
    print(f"{a.steps} steps: span {span / 1e3:.1f} us/step; compute stream = {comp}")
    by = {}
    for r in win:
        by.setdefault(r[3], []).append(r)
    for sid, rs in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy = union([(r[0], r[1]) for r in rs]) / a.steps
        print(f"  stream {sid:>4}: {len(rs) / a.steps:6.1f} kernels/step, busy {busy / 1e3:8.1f} us/step "
              f"({100 * busy / span:5.1f} % of the span)")
    # forward / backward split of each step on the compute stream, and the compute stream's gaps
    cs = [r for r in win if r[3] == comp]
    gaps = {}
    fwd_t, bwd_t, fwd_busy, bwd_busy = 0, 0, 0, 0
    step_ends = [rows[i][1] for i in ends[-a.steps - 1:]]
    for k in range(a.steps):
        s0, s1 = step_ends[k], step_ends[k + 1]
        st = [r for r in cs if s0 <= r[0] < s1 + 1]
        if not st:
            continue
        li = [i for i, r in enumerate(st) if a.loss_kernel in r[2]]
        cut = st[li[0]][1] if li else st[-1][1]
        fwd = [r for r in st if r[0] < cut]
        bwd = [r for r in st if r[0] >= cut]
        if fwd:
            fwd_t += fwd[-1][1] - fwd[0][0]
            fwd_busy += union([(r[0], r[1]) for r in fwd])
        if bwd:
            bwd_t += bwd[-1][1] - bwd[0][0]
            bwd_busy += union([(r[0], r[1]) for r in bwd])
        last_e, last_n = st[0][1], st[0][2]
        for r in st[1:]:
            if r[0] > last_e:
                key = (short(last_n), short(r[2]))
                t, c = gaps.get(key, (0, 0))
                gaps[key] = (t + r[0] - last_e, c + 1)
            if r[1] > last_e:
                last_e, last_n = r[1], r[2]
    n = a.steps
    print(f"compute stream forward: {fwd_t / n / 1e3:.1f} us/step wall, {fwd_busy / n / 1e3:.1f} busy; "
          f"backward: {bwd_t / n / 1e3:.1f} us/step wall, {bwd_busy / n / 1e3:.1f} busy")
    tot = sum(t for t, _ in gaps.values())
    print(f"compute-stream idle inside the steps: {tot / n / 1e3:.1f} us/step; largest (previous -> next kernel):")
    for (p, q), (t, c) in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:a.gaps]:
        print(f"  {t / n / 1e3:8.1f} us/step  n/step={c / n:5.1f}  {p}  ->  {q}")


if __name__ == "__main__":
    main()
