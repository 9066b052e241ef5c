#!/bin/bash
# Round-4 shipped-build evidence (one GPU): bench + rocprof per-step tables (ResNet-50, BERT-base),
# serial layer profile, secondary benchmark suite (hip only).  Outputs under gpurun_out/r4f_*.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/r4f_bench.txt 2>&1 || { tail -20 gpurun_out/r4f_bench.txt; exit 1; }
tail -1 gpurun_out/r4f_bench.txt | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_bench.log 2>&1 || { echo "bench rocprof failed"; tail -30 gpurun_out/prof_bench.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bench --top 60 --last-steps 4 > gpurun_out/r4f_prof_bench.txt
find gpurun_out/prof_bench -name "*kernel_trace.csv" -delete
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o run -- python tools/prof_target.py bert 16 > gpurun_out/prof_bert.log 2>&1 || { echo "bert rocprof failed"; tail -30 gpurun_out/prof_bert.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bert --top 45 --step-kernel adam_flat --last-steps 4 > gpurun_out/r4f_prof_bert.txt
find gpurun_out/prof_bert -name "*kernel_trace.csv" -delete
PCMP_WGRAD_STREAM=0 timeout -k 10 300 python tools/layer_profile.py --top 60 > gpurun_out/r4f_layer_profile.txt 2>&1 || { echo "layer profile failed"; tail -20 gpurun_out/r4f_layer_profile.txt; exit 1; }
SUITE_HIP_ONLY=1 timeout -k 10 600 python -u tools/bench_suite.py > gpurun_out/r4f_bench_suite.txt 2>&1 || { echo "suite failed"; tail -20 gpurun_out/r4f_bench_suite.txt; exit 1; }
cat gpurun_out/r4f_bench_suite.txt | grep "^{" | cut -c1-200
