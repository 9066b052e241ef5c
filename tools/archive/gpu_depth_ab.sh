#!/bin/bash
# Run-ahead depth A/B (PCMP_MAX_INFLIGHT=1 vs 2), interleaved, ResNet-50 and ResNet-18 -> gpurun_out/depth_ab.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/depth_ab.log
run() { echo "== depth $PCMP_MAX_INFLIGHT $*" >> $L; timeout -k 10 300 python bench.py "$@" >> $L 2>&1; }
for r in 1 2 3; do
  for d in 2 1; do
    PCMP_MAX_INFLIGHT=$d run --steps 30 --warmup 5 || { tail -20 $L; exit 1; }
  done
done
for d in 2 1; do PCMP_MAX_INFLIGHT=$d run --steps 50 --warmup 5 --model resnet18 || { tail -20 $L; exit 1; }; done
grep -E '^==|^\{' $L | cut -c1-110
