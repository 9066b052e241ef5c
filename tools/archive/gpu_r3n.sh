#!/bin/bash
# BatchNorm-backward fold (PCMP_DZ_FOLD): kernel + model tests, then whole-step ResNet-50 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fold" > gpurun_out/r3n_fold_tests.log 2>&1 || { echo fold tests failed; tail -40 gpurun_out/r3n_fold_tests.log; exit 1; }
tail -2 gpurun_out/r3n_fold_tests.log
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_models_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
out=gpurun_out/r3n_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_DZ_FOLD=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3n_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3n_b.log; exit 1; }
    echo "round $r dz_fold=$v $(tail -1 gpurun_out/r3n_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
