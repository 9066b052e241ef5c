#!/bin/bash
# Current-build evidence: steady-state rocprofv3 per-step kernel table (ResNet-50 B=256), a per-op
# layer profile with the WGRAD side stream off (event brackets are exact only without concurrency),
# and the HW-queue setting the box exports.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-<unset>}"
TAG=${TAG:-r2c}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_$TAG.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_$TAG --top 60 --last-steps 4 > gpurun_out/prof_${TAG}_summary.txt
sed -n '/per step over/,$p' gpurun_out/prof_${TAG}_summary.txt | head -40
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -delete
PCMP_WGRAD_STREAM=0 timeout -k 10 300 python tools/layer_profile.py --model resnet50 --batch 256 --top 70 > gpurun_out/layer_profile_serial.txt 2>&1 || { echo "layer profile failed"; tail -20 gpurun_out/layer_profile_serial.txt; exit 1; }
head -25 gpurun_out/layer_profile_serial.txt
