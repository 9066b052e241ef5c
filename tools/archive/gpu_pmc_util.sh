#!/bin/bash
# MFMA / LDS utilisation of single conv microbench cases (one rocprofv3 --pmc pass each):
# CASES="shape:mode shape:mode ..."  -> gpurun_out/pmc_util.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
CTRS="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for c in ${CASES:-l3_3x3_256:fwd l2_3x3_128:fwd l1_3x3_64:fwd l3_3x3_256:wgrad}; do
  sh=${c%%:*}; md=${c##*:}
  d=gpurun_out/pmcu_${sh}_${md}
  timeout -s KILL 90 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $d -o run -- python tools/conv_micro.py --iters 2 --only $sh --modes $md > $d.log 2>&1 || { echo "pmc $c failed"; tail -5 $d.log; exit 1; }
done
python tools/pmc_util_summary.py gpurun_out/pmcu_* > gpurun_out/pmc_util.txt
cat gpurun_out/pmc_util.txt
