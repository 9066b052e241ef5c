#!/bin/bash
# BERT fusion round: fused-op kernel tests, then fused vs op-by-op BERT-base step (eager + hipGraph),
# then a kernel profile of the fused graphed step.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_text_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
out=gpurun_out/r3i_ab.txt; : > $out
for r in 1 2; do
  for v in 0 1; do
    PCMP_BERT_FUSED=$v SUITE_HIP_ONLY=1 timeout -k 10 300 python -u tools/bench_suite.py bert_train > gpurun_out/r3i_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3i_b.log; exit 1; }
    grep bert_train gpurun_out/r3i_b.log | sed "s/^/round $r fused=$v /" | tee -a $out
  done
done
SUITE_HIP_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o run -- python tools/bench_suite.py bert_train > gpurun_out/prof_bert.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_bert.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bert --top 45 > gpurun_out/prof_bert_summary.txt
head -60 gpurun_out/prof_bert_summary.txt
find gpurun_out/prof_bert -name "*kernel_trace.csv" -delete; true
