#!/bin/bash
# Whole-step A/B: high-priority compute stream (PCMP_STEP_PRIO) and early-prefetch DMA schedule
# (dma_pf2, race-fixed), interleaved rounds; BERT eager vs hipGraph.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r3f_ab.txt; : > $out
for r in 1 2 3; do
  for v in base prio pf2 prio_pf2; do
    case $v in base) E="";; prio) E="PCMP_STEP_PRIO=1";; pf2) E="PCMP_KNOBS=dma_pf2=3";; prio_pf2) E="PCMP_STEP_PRIO=1 PCMP_KNOBS=dma_pf2=3";; esac
    env $E timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3f_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3f_b.log; exit 1; }
    echo "round $r $v $(tail -1 gpurun_out/r3f_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
SUITE_HIP_ONLY=1 timeout -k 10 300 python tools/bench_suite.py bert_train > gpurun_out/r3f_bert.txt 2>&1 || { echo bert failed; tail -20 gpurun_out/r3f_bert.txt; exit 1; }
cat gpurun_out/r3f_bert.txt | grep bench
