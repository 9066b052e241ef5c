#!/bin/bash
# Iteration loop on the GPU box: selected GPU tests -> flagship bench -> per-op layer profile.
# TESTS (default: kernel + model numerics), BENCH_ARGS, PROFILE=0 to skip the layer profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-"tests/test_kernels_gpu.py tests/test_models_gpu.py"}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/iter_tests.log; exit 1; }
tail -2 gpurun_out/iter_tests.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/iter_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/iter_bench.log; exit 1; }
tail -1 gpurun_out/iter_bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  PCMP_WGRAD_STREAM=0 timeout -k 10 300 python tools/layer_profile.py > gpurun_out/iter_layer_profile.txt 2>&1 || { echo "layer profile failed"; tail -20 gpurun_out/iter_layer_profile.txt; exit 1; }
  head -22 gpurun_out/iter_layer_profile.txt
fi
