#!/bin/bash
# Large per-GPU batch investigation: bench at B=512/768 with allocator statistics, then a
# rocprofv3 kernel-trace summary at B=768 -> gpurun_out/bigbatch.log, gpurun_out/prof_summary_b768.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PCMP_MEMSTATS=1
for B in 512 768; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 3 --batch-size $B >> gpurun_out/bigbatch.log 2>&1 || { echo "bench B=$B failed"; tail -20 gpurun_out/bigbatch.log; exit 1; }
done
grep -E '^\{|\[bench\] mem' gpurun_out/bigbatch.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof768 -o run -- python bench.py --steps 3 --warmup 2 --batch-size 768 > gpurun_out/prof768.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof768.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof768 --steps 5 --top 30 > gpurun_out/prof_summary_b768.txt
cat gpurun_out/prof_summary_b768.txt
find gpurun_out/prof768 -name "*kernel_trace.csv" -delete; true
