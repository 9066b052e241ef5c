#!/bin/bash
# rocprofv3 kernel trace of the batch-1 hipGraph inference loop (tools/prof_infer.py): per-image
# kernel count / span / busy and the kernel timeline of one steady-state image.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inf -o run -- python tools/prof_infer.py 200 > gpurun_out/prof_inf.log 2>&1 || { tail -20 gpurun_out/prof_inf.log; exit 1; }
grep p50 gpurun_out/prof_inf.log
python tools/prof_summary.py gpurun_out/prof_inf --top 30 --last-steps 0 > gpurun_out/r4_prof_infer_summary.txt
python - >> gpurun_out/r4_prof_infer_summary.txt <<'PY'
import csv, glob, statistics
f = glob.glob("gpurun_out/prof_inf/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
groups, cur = [], [ts[0]]
for a, b in zip(ts, ts[1:]):
    if b[0] - max(x[1] for x in cur[-8:]) > 20000:
        groups.append(cur); cur = []
    cur.append(b)
groups.append(cur)
groups = [g for g in groups if len(g) > 20][-100:]
span = [(max(e for _, e, _ in g) - g[0][0]) / 1e3 for g in groups]
nk = [len(g) for g in groups]
print(f"per inference: kernels {statistics.median(nk)}, GPU span {statistics.median(span):.1f} us")
g = groups[len(groups) // 2]
t0, last_end = g[0][0], g[0][0]
print("one image's kernels: start / dur / gap-after-latest-end (us)")
for s, e, n in g:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {(s - last_end) / 1e3:7.1f}  {n[:110]}")
    last_end = max(last_end, e)
PY
find gpurun_out/prof_inf -name "*kernel_trace.csv" -delete
head -5 gpurun_out/r4_prof_infer_summary.txt
