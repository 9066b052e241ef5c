#!/bin/bash
# Instruction mix (VALU / MFMA / SALU / LDS / VMEM) of single conv microbench cases, one pass each:
# CASES="shape:mode ..." -> gpurun_out/pmc_mix.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CTRS="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for c in ${CASES:-l3_3x3_256:wgrad l1_3x3_64:wgrad l3_3x3_256:fwd l2_3x3_128:fwd}; do
  sh=${c%%:*}; md=${c##*:}
  d=gpurun_out/pmcm_${sh}_${md}
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $d -o run -- python tools/conv_micro.py --iters 2 --only $sh --modes $md > $d.log 2>&1 || { echo "pmc $c failed"; tail -5 $d.log; exit 1; }
done
python - <<'PY' > gpurun_out/pmc_mix.txt
import csv, glob, os, collections
for d in sorted(glob.glob("gpurun_out/pmcm_*")):
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
        mf = c["SQ_INSTS_MFMA"] or 1
        print(f"   {k:60s} VALU/MFMA {c['SQ_INSTS_VALU'] / mf:6.2f}  SALU/MFMA {c['SQ_INSTS_SALU'] / mf:5.2f}  "
              f"LDS/MFMA {c['SQ_INSTS_LDS'] / mf:5.2f}  VMEM/MFMA {c['SQ_INSTS_VMEM_RD'] / mf:5.2f}  "
              f"MFMA-busy/GUI {c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1, c['GRBM_GUI_ACTIVE']):7.2f}  "
              f"VALU-active/GUI {c['SQ_ACTIVE_INST_VALU'] / max(1, c['GRBM_GUI_ACTIVE']):7.2f}")
PY
cat gpurun_out/pmc_mix.txt
