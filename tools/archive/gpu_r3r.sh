#!/bin/bash
# WGRAD DMA per-shape policy (wgrad_dma=2) vs register-staged (0): WGRAD tests + whole-step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PCMP_KNOBS=wgrad_dma=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/r3r_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
out=gpurun_out/r3r_ab.txt; : > $out
for r in 1 2 3 4; do
  for v in 0 2; do
    PCMP_KNOBS=wgrad_dma=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3r_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3r_b.log; exit 1; }
    echo "round $r wgrad_dma=$v $(tail -1 gpurun_out/r3r_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
