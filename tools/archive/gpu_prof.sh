#!/bin/bash
# rocprofv3 kernel-trace/stats of the flagship bench (7 steps: 2 warmup + 5 timed) -> gpurun_out/prof_summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 2"}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py $ARGS > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof --steps ${PROF_STEPS:-7} --top 45 > gpurun_out/prof_summary.txt
cat gpurun_out/prof_summary.txt
rm -rf gpurun_out/prof/*/*.csv.bak 2>/dev/null; find gpurun_out/prof -name "*kernel_trace.csv" -delete; true
