#!/bin/bash
# Instruction mix (VALU / MFMA / SALU / LDS / VMEM) of single conv microbench cases, one pass each:
# CASES="shape:mode ..." -> gpurun_out/pmc_wait.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CTRS="SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for c in ${CASES:-l3_3x3_256:wgrad l1_3x3_64:wgrad l3_3x3_256:fwd l2_3x3_128:fwd}; do
  sh=${c%%:*}; md=${c##*:}
  d=gpurun_out/pmcw_${sh}_${md}
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $d -o run -- python tools/conv_micro.py --iters 2 --only $sh --modes $md > $d.log 2>&1 || { echo "pmc $c failed"; tail -5 $d.log; exit 1; }
done
python - <<'PY' > gpurun_out/pmc_wait.txt
import csv, glob, os, collections
for d in sorted(glob.glob("gpurun_out/pmcw_*")):
    if not os.path.isdir(d):
        continue
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if "igemm" not in r["Kernel_Name"]:
            continue
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    print(os.path.basename(d))
    for k, c in agg.items():
        wc = c["SQ_WAVE_CYCLES"] or 1
        print(f"   {k:60s} wait-LDS-issue {c['SQ_WAIT_INST_LDS'] / wc:5.2f}  wait-issue-any {c['SQ_WAIT_INST_ANY'] / wc:5.2f}  "
              f"wait-any(waitcnt/barrier) {c['SQ_WAIT_ANY'] / wc:5.2f}  LDS-active/GUI {c['SQ_LDS_IDX_ACTIVE'] / max(1, c['GRBM_GUI_ACTIVE']):7.2f}  "
              f"LDS-inst-active/wave-cyc {c['SQ_ACTIVE_INST_LDS'] / wc:5.2f}")
PY
cat gpurun_out/pmc_wait.txt
