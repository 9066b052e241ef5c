set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1 || true
grep -oE "TCC_EA0?_[A-Z0-9_]+|TCC_[A-Z_]*WR[A-Z0-9_]*|TCP_[A-Z_]*" gpurun_out/pmc_list.txt | sort -u | head -80
for w in fwd fill; do
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum -d gpurun_out/pmc_$w -o run --output-format csv -- python tools/pmc_probe_fwd.py $w > gpurun_out/pmc_$w.log 2>&1 || { echo "pmc $w failed"; tail -5 gpurun_out/pmc_$w.log; }
find gpurun_out/pmc_$w -name "*counter_collection.csv" | head -1 | xargs -I{} sh -c 'python3 - {} <<"PY"
import csv,sys,collections
d=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k=(r["Kernel_Name"][:60], r["Counter_Name"]); d[k]+=float(r["Counter_Value"]); n[k]+=1
for k,v in sorted(d.items()): print(k, v/ max(1,n[k]) * 0 + v)
PY'
done
