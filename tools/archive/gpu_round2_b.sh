#!/bin/bash
# Full GPU test suite, bench, secondary suite (BERT / BiLSTM / ResNet-18 / batch-1) and a BERT
# rocprofv3 kernel summary (checks that no hipBLASLt / rocBLAS kernel runs).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 600 python -u tools/bench_suite.py ${SUITE:-bert_train bilstm_train resnet18_train resnet50_infer} > gpurun_out/suite.log 2>&1 || { echo suite failed; tail -20 gpurun_out/suite.log; exit 1; }
grep '^{' gpurun_out/suite.log
SUITE_HIP_ONLY=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o run -- python tools/bench_suite.py bert_train > gpurun_out/prof_bert.log 2>&1 || { echo rocprof failed; tail -20 gpurun_out/prof_bert.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bert --top 40 --last-steps 0 > gpurun_out/prof_bert_summary.txt
head -42 gpurun_out/prof_bert_summary.txt
echo "blas kernels: $(grep -ciE 'Cijk|hipblaslt|rocblas|gemm_kernel' gpurun_out/prof_bert_summary.txt || true)"
find gpurun_out/prof_bert -name "*kernel_trace.csv" -delete; true
