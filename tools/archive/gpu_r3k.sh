#!/bin/bash
# attention forward v2 (register-resident) vs v1: text kernel tests, BERT step A/B, kernel times.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_text_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3k_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3k_tests.log; exit 1; }
tail -2 gpurun_out/r3k_tests.log
out=gpurun_out/r3k_ab.txt; : > $out
for r in 1 2; do
  for v in 1 0; do
    PCMP_ATTN_BWD_V1=$v SUITE_HIP_ONLY=1 timeout -k 10 300 python -u tools/bench_suite.py bert_train > gpurun_out/r3k_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3k_b.log; exit 1; }
    grep bert_train gpurun_out/r3k_b.log | sed "s/^/round $r attn_bwd_v1=$v /" | tee -a $out
  done
done
SUITE_HIP_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert3 -o run -- python tools/bench_suite.py bert_train > gpurun_out/prof_bert3.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_bert3.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bert3 --top 45 > gpurun_out/prof_bert3_summary.txt
grep -E "attention|ln_bwd|layernorm" gpurun_out/prof_bert3_summary.txt
find gpurun_out/prof_bert3 -name "*kernel_trace.csv" -delete; true
