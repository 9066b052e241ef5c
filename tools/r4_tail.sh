#!/bin/bash
# End-of-backward tail of the flagship step (tools/tail_report.py over a rocprofv3 kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tail -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_tail.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_tail.log; exit 1; }
python tools/tail_report.py gpurun_out/prof_tail --steps 3 --last 24 > gpurun_out/r4_tail.txt 2>&1
find gpurun_out/prof_tail -name "*kernel_trace.csv" -delete
head -40 gpurun_out/r4_tail.txt
