#!/bin/bash
# batch-1 in-graph D2H A/B + kernel timeline (queue / stream ids) around the loss -> backward boundary
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/b1_hostout_ab.py > gpurun_out/b1_hostout_ab.txt 2>&1 || { echo "b1 ab failed"; tail -20 gpurun_out/b1_hostout_ab.txt; exit 1; }
cat gpurun_out/b1_hostout_ab.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_around -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_around.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_around.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_around --top 5 --last-steps 0 --around xent_grad_scale --around-n 16 > gpurun_out/around_xent.txt
python tools/prof_summary.py gpurun_out/prof_around --top 5 --last-steps 0 --around sgd_flat --around-n 16 > gpurun_out/around_sgd.txt
sed -n '/timeline/,$p' gpurun_out/around_xent.txt gpurun_out/around_sgd.txt
find gpurun_out/prof_around -name "*kernel_trace.csv" -delete
