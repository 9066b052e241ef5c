#!/bin/bash
# LDS-DMA WGRAD: kernel tests, shape-level A/B, whole-step ResNet-50 and BERT A/B (wgrad_dma 0/1).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_text_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3l_tests.log; exit 1; }
tail -2 gpurun_out/r3l_tests.log
timeout -k 10 400 python -u tools/gemm_knob_ab.py --variants 'reg:wgrad_dma=0;dma:wgrad_dma=1' --modes wgrad --rounds 3 > gpurun_out/r3l_shape_ab.txt 2>&1 || { echo knob failed; tail -20 gpurun_out/r3l_shape_ab.txt; exit 1; }
cat gpurun_out/r3l_shape_ab.txt
out=gpurun_out/r3l_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_KNOBS=wgrad_dma=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3l_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3l_b.log; exit 1; }
    echo "round $r wgrad_dma=$v $(tail -1 gpurun_out/r3l_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
for v in 0 1; do
  PCMP_KNOBS=wgrad_dma=$v SUITE_HIP_ONLY=1 timeout -k 10 300 python -u tools/bench_suite.py bert_train > gpurun_out/r3l_bb.log 2>&1 || { echo "bert $v failed"; tail -20 gpurun_out/r3l_bb.log; exit 1; }
  grep bert_train gpurun_out/r3l_bb.log | sed "s/^/wgrad_dma=$v /" | tee -a $out
done
