#!/bin/bash
# s2d kernel timing + its test, batch-1 inference kernel profile, flagship bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "s2d" > gpurun_out/s2d_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/s2d_tests.log; exit 1; }
tail -1 gpurun_out/s2d_tests.log
timeout -k 10 120 python tools/s2d_time.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_e.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_e.log; exit 1; }
tail -1 gpurun_out/bench_e.log
bash tools/gpu_prof_infer.sh
