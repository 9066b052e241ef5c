#!/bin/bash
# Batched WGRAD side-stream fork A/B (PCMP_WGRAD_BATCH=0/1), interleaved, plus model GPU tests
# with batching on -> gpurun_out/wbatch_ab.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/wbatch_ab.log
PCMP_WGRAD_BATCH=1 timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread >> $L 2>&1 || { tail -30 $L; exit 1; }
run() { echo "== $*" >> $L; timeout -k 10 300 "$@" >> $L 2>&1; }
for r in 1 2; do
  PCMP_WGRAD_BATCH=0 run python bench.py --steps 30 --warmup 5 || { tail -20 $L; exit 1; }
  PCMP_WGRAD_BATCH=1 run python bench.py --steps 30 --warmup 5 || { tail -20 $L; exit 1; }
done
PCMP_WGRAD_BATCH=0 run python bench.py --steps 30 --warmup 5 --model resnet18 || { tail -20 $L; exit 1; }
PCMP_WGRAD_BATCH=1 run python bench.py --steps 30 --warmup 5 --model resnet18 || { tail -20 $L; exit 1; }
grep -E 'passed|failed|^\{' $L | cut -c1-130
