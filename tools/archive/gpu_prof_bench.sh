#!/bin/bash
# Bench + steady-state rocprofv3 per-step kernel table of the flagship (ResNet-50 B=256).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-cur}
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_$TAG.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_$TAG --top 60 --last-steps 4 > gpurun_out/prof_${TAG}_summary.txt
sed -n '/per step over/,$p' gpurun_out/prof_${TAG}_summary.txt | head -64
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete; true
