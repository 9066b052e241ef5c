#!/bin/bash
# BERT iteration on one GPU: text-path GPU tests, GEMM / attention micro benchmarks, whole-step A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_text_f32_gpu.py tests/test_text_kernels_gpu.py} > gpurun_out/r4_bert_tests.log 2>&1 || { tail -30 gpurun_out/r4_bert_tests.log; exit 1; }
tail -2 gpurun_out/r4_bert_tests.log
timeout -k 10 300 python -u tools/bert_gemm_micro.py --rounds 3 > gpurun_out/r4_bert_gemm_micro.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_micro.py > gpurun_out/r4_attn_micro.txt 2>&1 || exit 1
cat gpurun_out/r4_bert_gemm_micro.txt gpurun_out/r4_attn_micro.txt
timeout -k 10 600 python -u tools/bert_ab.py --variants "${VARIANTS:-serial:PCMP_WGRAD_STREAM=0;side:}" --rounds 3 > gpurun_out/r4_bert_ab.txt 2>&1 || exit 1
cat gpurun_out/r4_bert_ab.txt
