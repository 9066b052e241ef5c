#!/bin/bash
# Staggered 8-wave schedule: correctness tests, plain-GEMM + conv-shape A/B, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dma8_staggered or loss_mean or conv_fwd" > gpurun_out/r3b_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
timeout -k 10 240 python -u tools/gemm_probe.py --rounds 3 --variants 'lock:dma8_stag=0;stag:dma8_stag=1' > gpurun_out/r3b_gemm_probe.txt 2>&1 || { echo probe failed; tail -20 gpurun_out/r3b_gemm_probe.txt; exit 1; }
cat gpurun_out/r3b_gemm_probe.txt
timeout -k 10 300 python -u tools/gemm_knob_ab.py --variants 'lock:dma8_stag=0;stag:dma8_stag=1' --modes fwd,dgrad --only l3_3x3,l3_1x1,l4_,l2_3x3 --rounds 3 > gpurun_out/r3b_shape_ab.txt 2>&1 || { echo knob failed; tail -20 gpurun_out/r3b_shape_ab.txt; exit 1; }
cat gpurun_out/r3b_shape_ab.txt
for v in 0 1 0 1; do PCMP_KNOBS=dma8_stag=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --infer-images 0 > gpurun_out/r3b_bench_$v.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r3b_bench_$v.log; exit 1; }; echo "stag=$v $(tail -1 gpurun_out/r3b_bench_$v.log | cut -c1-140)"; done
