#!/bin/bash
# Early-prefetch (dma_pf2) schedule: bitwise tests, plain GEMM + conv-shape A/B, whole-step A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dma8_staggered or dma4_early or resize" > gpurun_out/r3d_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r3d_tests.log; exit 1; }
tail -2 gpurun_out/r3d_tests.log
timeout -k 10 240 python -u tools/gemm_probe.py --rounds 3 --no-blas --variants 'lock:;pf2:dma_pf2=3;stag:dma8_stag=1' > gpurun_out/r3d_gemm_probe.txt 2>&1 || { echo probe failed; tail -20 gpurun_out/r3d_gemm_probe.txt; exit 1; }
cat gpurun_out/r3d_gemm_probe.txt
timeout -k 10 400 python -u tools/gemm_knob_ab.py --variants 'lock:;pf2:dma_pf2=3' --modes fwd,dgrad --rounds 3 > gpurun_out/r3d_shape_ab.txt 2>&1 || { echo knob failed; tail -20 gpurun_out/r3d_shape_ab.txt; exit 1; }
cat gpurun_out/r3d_shape_ab.txt
for v in 0 3 0 3; do PCMP_KNOBS=dma_pf2=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --infer-images 0 > gpurun_out/r3d_bench_$v.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r3d_bench_$v.log; exit 1; }; echo "pf2=$v $(tail -1 gpurun_out/r3d_bench_$v.log | cut -c1-120)"; done
