#!/bin/bash
# Whole-step hipGraph A/B: eager vs --graph, same total step count (graph mode spends 2 warm-up
# steps + 1 replay inside graph_step), so final losses must be bitwise equal (deterministic kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in ${MODELS:-resnet50 resnet18}; do
  timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/ga_${m}_eager.log 2>&1 || { echo "eager $m failed"; tail -20 gpurun_out/ga_${m}_eager.log; exit 1; }
  tail -1 gpurun_out/ga_${m}_eager.log
  timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 2 --graph > gpurun_out/ga_${m}_graph.log 2>&1 || { echo "graph $m failed"; tail -20 gpurun_out/ga_${m}_graph.log; exit 1; }
  tail -1 gpurun_out/ga_${m}_graph.log
done
