#!/bin/bash
# SQ counters of the halo kernel vs the implicit GEMM on the layer-1 3x3 FWD
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+" gpurun_out/pmc_list.txt | sort -u | tr '\n' ' ' | head -c 6000; echo
summ() { find $1 -name "*counter_collection.csv" | head -1 | xargs -I{} python3 -c '
import csv,sys,collections
d=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "halo" not in r["Kernel_Name"] and "igemm" not in r["Kernel_Name"]: continue
    k=(r["Kernel_Name"][:50], r["Counter_Name"]); d[k]+=float(r["Counter_Value"]); n[k]+=1
for k,v in sorted(d.items()): print(k, "%.4g" % (v / n[k]))
' {}; }
for h in 0 1; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_LDS -d gpurun_out/pmch_$h -o run --output-format csv -- python tools/pmc_halo.py $h > gpurun_out/pmch_$h.log 2>&1 || { echo "pmc $h failed"; tail -5 gpurun_out/pmch_$h.log; exit 1; }
echo "== halo=$h"; summ gpurun_out/pmch_$h
done
