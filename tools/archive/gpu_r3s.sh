#!/bin/bash
# round-3 rocprof stats of the flagship step + end-of-backward tail report
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3s -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_r3s.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_r3s.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_r3s --top 60 --last-steps 4 > gpurun_out/prof_r3s_summary.txt
python tools/tail_report.py gpurun_out/prof_r3s --steps 3 --last 24 > gpurun_out/r3s_tail.txt
python tools/queue_report.py gpurun_out/prof_r3s > gpurun_out/r3s_queues.txt || true
cat gpurun_out/r3s_tail.txt
sed -n '/per step over/,$p' gpurun_out/prof_r3s_summary.txt | head -30
find gpurun_out/prof_r3s -name "*kernel_trace.csv" -delete; true
