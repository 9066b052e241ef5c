#!/bin/bash
# EPI_GELU split: GEMM/GELU tests, batch-1 inference + BERT + ResNet-50 numbers, batch-1 rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_text_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3y_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3y_tests.log; exit 1; }
tail -1 gpurun_out/r3y_tests.log
for r in 1 2; do
  SUITE_HIP_ONLY=1 timeout -k 10 300 python -u tools/bench_suite.py resnet50_infer bert_train > gpurun_out/r3y.log 2>&1 || { echo "suite failed"; tail -20 gpurun_out/r3y.log; exit 1; }
  grep -E '"hip\+graph"|"bert_train", "impl": "hip"' gpurun_out/r3y.log | cut -c1-140
done
timeout -k 10 200 python bench.py > gpurun_out/r3y_b.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r3y_b.log; exit 1; }
tail -1 gpurun_out/r3y_b.log | cut -c1-200
bash tools/gpu_prof_infer.sh > gpurun_out/r3y_infer_prof.txt 2>&1 || { echo infer prof failed; tail -20 gpurun_out/r3y_infer_prof.txt; exit 1; }
grep -E "p50|per inference" gpurun_out/r3y_infer_prof.txt
head -8 gpurun_out/prof_inf_summary.txt | cut -c1-120
find gpurun_out/prof_inf -name "*kernel_trace.csv" -delete; true
