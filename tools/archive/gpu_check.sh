#!/bin/bash
# GPU verification: kernel + model numerics, conv microbench vs MIOpen, flagship bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q > gpurun_out/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python tools/conv_micro.py --torch > gpurun_out/micro.log 2>&1 || { echo "micro failed"; tail -20 gpurun_out/micro.log; exit 1; }
grep -v Warn gpurun_out/micro.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$SUITE" ]; then
  timeout -k 10 400 python tools/bench_suite.py $SUITE > gpurun_out/suite.log 2>&1 || { echo "suite failed"; tail -20 gpurun_out/suite.log; exit 1; }
  grep '^{' gpurun_out/suite.log
fi
