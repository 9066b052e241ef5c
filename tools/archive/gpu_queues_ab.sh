#!/bin/bash
# HW-queue count A/B: plain vs forced-RCCL bench at GPU_MAX_HW_QUEUES=4 and 8, plus a short trace
# of each forced arm to read which queue each stream's kernels ran on.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # $1 = label, $2 = queues, rest = bench args
  local lab=$1 q=$2; shift 2
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 5 --infer-images 0 "$@" > gpurun_out/q_$lab.log 2>&1 || { echo "bench $lab failed"; tail -30 gpurun_out/q_$lab.log; exit 1; }
  echo "$lab $(grep '^{' gpurun_out/q_$lab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  run plain_q4_$r 4 || exit 1
  run plain_q8_$r 8 || exit 1
  run force_q4_$r 4 --ddp-force || exit 1
  run force_q8_$r 8 --ddp-force || exit 1
done
for q in 4 8; do
  for arm in plain force; do
    extra=""; [ $arm = force ] && extra="--ddp-force"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_q${q}_$arm -o run -- python bench.py --steps 3 --warmup 2 --infer-images 0 $extra > gpurun_out/prof_q${q}_$arm.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_q${q}_$arm.log; exit 1; }
  done
done
echo done
