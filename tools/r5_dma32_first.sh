#!/bin/bash
# Round-5 first GPU pass for igemm_dma32_kernel: numerics, per-shape A/B, whole-step A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dma32_gpu.py \
  tests/test_kernels_gpu.py tests/test_text_f32_gpu.py tests/test_text_kernels_gpu.py -k "dma32 or large_shapes or bn_reduce or conv_dgrad or conv_fwd or dropout or attention" > gpurun_out/r5_t1.log 2>&1 || { tail -40 gpurun_out/r5_t1.log; exit 1; }
tail -3 gpurun_out/r5_t1.log
timeout -k 10 600 python -u tools/gemm_knob_ab.py --variants 'new:dma32=1;old:dma32=0' --modes fwd,dgrad --rounds 3 \
  > gpurun_out/r5_knob_dma32.txt 2>&1 || { tail -20 gpurun_out/r5_knob_dma32.txt; exit 1; }
cat gpurun_out/r5_knob_dma32.txt
VARIANTS="new=dma32=1;old=dma32=0" ROUNDS=3 bash tools/r4_bench_ab.sh
