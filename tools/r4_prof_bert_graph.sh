#!/bin/bash
# rocprofv3 kernel trace of BERT-base GraphedStep replays (WGRAD side stream captured into the graph)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bg -o run -- python tools/prof_target.py bert_graph 12 > gpurun_out/prof_bg.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_bg.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bg --top 30 --step-kernel adam_flat --last-steps 3 --around adam_flat --around-n 40 > gpurun_out/r4_prof_bert_graph.txt
find gpurun_out/prof_bg -name "*kernel_trace.csv" -delete
head -80 gpurun_out/r4_prof_bert_graph.txt
