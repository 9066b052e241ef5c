set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inf -o run -- python tools/prof_infer.py 200 > gpurun_out/prof_inf.log 2>&1 || { tail -20 gpurun_out/prof_inf.log; exit 1; }
grep p50 gpurun_out/prof_inf.log
python tools/prof_summary.py gpurun_out/prof_inf --top 30 --last-steps 0 > gpurun_out/prof_inf_summary.txt
cat gpurun_out/prof_inf_summary.txt
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_inf/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# last 100 inferences: split on the argmax/graph-final kernel boundaries by gaps > 20 us
ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
groups, cur = [], [ts[0]]
for a, b in zip(ts, ts[1:]):
    if b[0] - a[1] > 20000:
        groups.append(cur); cur = []
    cur.append(b)
groups.append(cur)
groups = [g for g in groups if len(g) > 20][-100:]
import statistics
span = [ (g[-1][1] - g[0][0]) / 1e3 for g in groups]
busy = [ sum(e - s for s, e, _ in g) / 1e3 for g in groups]
nk = [len(g) for g in groups]
print(f"per inference: kernels {statistics.median(nk)}, GPU span {statistics.median(span):.1f} us, kernel busy {statistics.median(busy):.1f} us")
PY
find gpurun_out/prof_inf -name "*kernel_trace.csv" -delete
