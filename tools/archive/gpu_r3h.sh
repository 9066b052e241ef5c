#!/bin/bash
# Reference-config reruns at the reference's precision (fp32 on the HIP kernels) and at bf16, plus
# the steady-state rocprofv3 kernel table of the flagship step on the round-3 defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for dt in fp32 bf16; do
  PCMP_PHASE_TIMES=1 timeout -k 10 600 python -u pytorch_training_inference.py --models resnet50,vgg16 --dtype $dt --json gpurun_out/r3_repro_$dt.jsonl > gpurun_out/r3_repro_$dt.log 2>&1 || { echo "notebook flow $dt failed"; tail -40 gpurun_out/r3_repro_$dt.log; exit 1; }
  echo "== $dt"; grep -E "Epoch|Training time|Inference time|phase" gpurun_out/r3_repro_$dt.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3 -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_r3.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_r3.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_r3 --top 70 --last-steps 4 > gpurun_out/prof_r3_summary.txt
sed -n '/per step over/,$p' gpurun_out/prof_r3_summary.txt | head -30
find gpurun_out/prof_r3 -name "*kernel_trace.csv" -delete; true
