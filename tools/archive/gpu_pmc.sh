#!/bin/bash
# PMC counters (own run, kernel-trace only) for one conv microbench shape: ONLY=<shape> MODES=<fwd,...>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ONLY=${ONLY:-l1_1x1_64to256}
MODES=${MODES:-fwd}
i=0
for CTRS in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM" \
            "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d gpurun_out/pmc_$i -o run -- python tools/conv_micro.py --iters 2 --only $ONLY --modes $MODES > gpurun_out/pmc_$i.log 2>&1 || { echo "pmc $i failed"; tail -20 gpurun_out/pmc_$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_1 gpurun_out/pmc_2 gpurun_out/pmc_3
