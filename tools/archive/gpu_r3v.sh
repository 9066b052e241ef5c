#!/bin/bash
# BatchNorm-forward (activation) fold: kernel + model tests, whole-step A/B PCMP_ACT_FOLD 0/1
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "fold or stem or wgrad or conv_fwd or bottleneck or resnet" > gpurun_out/r3v_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3v_tests.log; exit 1; }
tail -1 gpurun_out/r3v_tests.log
out=gpurun_out/r3v_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_ACT_FOLD=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3v_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3v_b.log; exit 1; }
    echo "round $r act_fold=$v $(tail -1 gpurun_out/r3v_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
