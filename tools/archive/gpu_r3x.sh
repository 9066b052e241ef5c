#!/bin/bash
# batch-1 inference A/B: LDS-DMA early-prefetch schedule (dma_pf2) and the small-M split target
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r3x_infer_ab.txt; : > $out
for r in 1 2 3; do
  for k in "dma_pf2=3" "dma_pf2=0" "dma_pf2=2"; do
    PCMP_KNOBS=$k SUITE_HIP_ONLY=1 timeout -k 10 200 python -u tools/bench_suite.py resnet50_infer > gpurun_out/r3x.log 2>&1 || { echo "suite $k failed"; tail -20 gpurun_out/r3x.log; exit 1; }
    grep '"hip+graph"' gpurun_out/r3x.log | sed "s/^/round $r $k /" | tee -a $out
  done
done
