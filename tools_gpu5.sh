#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_text_kernels_gpu.py -q -m gpu -x > gpurun_out/text.log 2>&1; echo "text rc=$?" >> gpurun_out/text.log
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -m gpu > gpurun_out/tests5.log 2>&1; echo "tests rc=$?" >> gpurun_out/tests5.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench5.log 2>&1
tail -15 gpurun_out/text.log; tail -3 gpurun_out/tests5.log; tail -1 gpurun_out/bench5.log
