#!/bin/bash
# PMC passes on the 8-wave 256x256 DMA kernel (plain 8192^3 GEMM, lock-step vs staggered) and on
# hipBLASLt for the same GEMM: where does the matrix pipe idle?
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pmc3; export TMPDIR=/tmp
rocprofv3 --list-avail > gpurun_out/pmc3/avail.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for v in 0 1; do
  for pi in 1 2; do
    eval C=\$P$pi
    d=gpurun_out/pmc3/g8k_stag${v}_p$pi
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $d -o run -- python tools/gemm_one.py --plan 2 --knobs dma8_stag=$v > $d.log 2>&1 || { echo "pmc $d failed"; tail -5 $d.log; exit 1; }
  done
done
for pi in 1 2; do
  eval C=\$P$pi
  d=gpurun_out/pmc3/conv_l3_3x3_fwd_p$pi
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $d -o run -- python tools/gemm_one.py --conv l3_3x3_256:fwd_stats > $d.log 2>&1 || { echo "pmc $d failed"; tail -5 $d.log; exit 1; }
done
for g in g8k_stag0 g8k_stag1 conv_l3_3x3_fwd; do echo "== $g"; python tools/pmc_summary.py gpurun_out/pmc3/${g}_p1 gpurun_out/pmc3/${g}_p2; done > gpurun_out/pmc3/summary.txt 2>&1; cat gpurun_out/pmc3/summary.txt
find gpurun_out/pmc3 -name "*kernel_trace.csv" -delete; true
