#!/bin/bash
# rocprofv3 kernel stats of the BERT-base training step (tools/bench_suite.py bert_train, hip only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bilstm -o run -- python tools/prof_target.py bilstm > gpurun_out/prof_bilstm.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_bilstm.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bilstm --steps 13 --top 40 > gpurun_out/prof_bilstm_summary.txt
cat gpurun_out/prof_bilstm_summary.txt
find gpurun_out/prof_bilstm -name "*kernel_trace.csv" -delete
