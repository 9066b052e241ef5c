#!/bin/bash
# Numerics of the conv kernels, then A/B of the 4-wave LDS-DMA kernel (PCMP_DMA4) on the conv
# microbench, then the narrow-output tile choice (PCMP_DMA4_N64 1 vs 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dma4_kernels.log 2>&1 || { echo "kernel tests failed"; tail -40 gpurun_out/dma4_kernels.log; exit 1; }
tail -2 gpurun_out/dma4_kernels.log
VAR=PCMP_DMA4 A=0 B=1 MODES=fwd,dgrad,dgrad_bnr bash tools/gpu_ab_env.sh > gpurun_out/dma4_ab.txt 2>&1 || { cat gpurun_out/dma4_ab.txt; exit 1; }
cat gpurun_out/dma4_ab.txt
VAR=PCMP_DMA4_N64 A=1 B=2 MODES=fwd,dgrad,dgrad_bnr ONLY=l1_ bash tools/gpu_ab_env.sh > gpurun_out/dma4_n64_ab.txt 2>&1 || { cat gpurun_out/dma4_n64_ab.txt; exit 1; }
cat gpurun_out/dma4_n64_ab.txt
