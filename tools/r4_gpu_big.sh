#!/bin/bash
# Round-4 GEMM core check on one GPU: big-kernel numerics tests, then per-shape in-process A/B
# (tools/gemm_knob_ab.py, ResNet-50 B=256 conv shapes with their training epilogues) and plain-GEMM
# throughput (tools/gemm_probe.py).  Outputs under gpurun_out/r4_*.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_big_gemm_gpu.py \
  tests/test_text_f32_gpu.py > gpurun_out/r4_tests_big_f32.log 2>&1 || { tail -40 gpurun_out/r4_tests_big_f32.log; exit 1; }
tail -3 gpurun_out/r4_tests_big_f32.log
timeout -k 10 400 python -u tools/gemm_knob_ab.py --rounds 3 --modes fwd,dgrad \
  --variants 'base:;big:big=3,big_min256=1,big_min128=1;big128:big=2,big_min128=1' > gpurun_out/r4_knob_ab_big.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_probe.py --rounds 2 --no-blas --variants 'base:;big:big=3' > gpurun_out/r4_gemm_probe_big.txt 2>&1 || exit 1
cat gpurun_out/r4_knob_ab_big.txt gpurun_out/r4_gemm_probe_big.txt | tail -80
