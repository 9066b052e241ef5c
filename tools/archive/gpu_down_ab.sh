#!/bin/bash
# Model/DDP/engine GPU tests, then bench A/B of the downsample branch on the side stream (PCMP_DOWN_STREAM)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_ddp_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/down_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/down_tests.log; exit 1; }
tail -2 gpurun_out/down_tests.log
for v in 0 1 0 1; do
  PCMP_DOWN_STREAM=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/down_bench_$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/down_bench_$v.log; exit 1; }
  echo "PCMP_DOWN_STREAM=$v $(tail -1 gpurun_out/down_bench_$v.log | cut -c1-150)"
done
