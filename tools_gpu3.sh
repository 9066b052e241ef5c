#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -m gpu > gpurun_out/tests3.log 2>&1; echo "tests rc=$?" >> gpurun_out/tests3.log
timeout -k 10 300 python tools/grad_diag.py > gpurun_out/graddiag.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench3.log 2>&1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof3.log 2>&1; echo "prof rc=$?" >> gpurun_out/prof3.log
tail -4 gpurun_out/tests3.log; head -30 gpurun_out/graddiag.log; tail -1 gpurun_out/bench3.log
