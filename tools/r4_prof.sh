#!/bin/bash
# Round-4 attribution profiles on the shipped build (one GPU):
#   1. BERT-base B=32 S=128 train step: rocprofv3 kernel stats, steady-state per-step table (adam_flat ends a step)
#   2. ResNet-50 B=256 bench step: rocprofv3 kernel stats, per-step table over the last 4 steps
#   3. (LAYER=1) serial event-bracketed layer profile (tools/layer_profile.py, WGRAD side stream off)
# Outputs: gpurun_out/r4_prof_{bert,bench}_summary.txt, gpurun_out/r4_layer_profile.txt
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${BERT:-1}" = 1 ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o run -- python tools/prof_target.py bert 16 > gpurun_out/prof_bert.log 2>&1 || { echo "bert rocprof failed"; tail -30 gpurun_out/prof_bert.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bert --top 45 --step-kernel adam_flat --last-steps 4 > gpurun_out/r4_prof_bert_summary.txt
find gpurun_out/prof_bert -name "*kernel_trace.csv" -delete
sed -n '/per step over/,$p' gpurun_out/r4_prof_bert_summary.txt | head -40
fi
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_bench.log 2>&1 || { echo "bench rocprof failed"; tail -30 gpurun_out/prof_bench.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_bench --top 60 --last-steps 4 > gpurun_out/r4_prof_bench_summary.txt
find gpurun_out/prof_bench -name "*kernel_trace.csv" -delete
fi
if [ "${LAYER:-1}" = 1 ]; then
PCMP_WGRAD_STREAM=0 timeout -k 10 300 python tools/layer_profile.py --top 60 > gpurun_out/r4_layer_profile.txt 2>&1 || { echo "layer profile failed"; tail -20 gpurun_out/r4_layer_profile.txt; exit 1; }
head -30 gpurun_out/r4_layer_profile.txt
fi
