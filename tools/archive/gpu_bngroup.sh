#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_model_parity_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/kt.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
for g in 0 1 0 1; do
  PCMP_KNOBS=bn_group=$g timeout -k 10 300 python bench.py --steps 20 --warmup 5 --infer-images 0 > gpurun_out/bench_g$g.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_g$g.log; exit 1; }
  echo "bn_group=$g $(grep -o '"value": [0-9.]*' gpurun_out/bench_g$g.log)"
done
