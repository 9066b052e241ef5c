#!/bin/bash
# fused BERT embedding LayerNorm: kernel + model tests, then the step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_text_kernels_gpu.py tests/test_model_parity_gpu.py -x -q --timeout 120 --timeout-method thread -k "layernorm or bert or embed" > gpurun_out/bert_emb_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/bert_emb_tests.log; exit 1; }
tail -1 gpurun_out/bert_emb_tests.log
timeout -k 10 300 python tools/bert_emb_ab.py > gpurun_out/bert_emb_ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/bert_emb_ab.txt; exit 1; }
grep round gpurun_out/bert_emb_ab.txt
