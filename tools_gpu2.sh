#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_models_gpu.py -x -q -m gpu > gpurun_out/models.log 2>&1; echo "models rc=$?" >> gpurun_out/models.log
timeout -k 10 200 python tools/train_curve.py --impl hip > gpurun_out/curve.log 2>&1
timeout -k 10 200 python tools/train_curve.py --impl torch >> gpurun_out/curve.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof1.log 2>&1; echo "prof rc=$?" >> gpurun_out/prof1.log
tail -5 gpurun_out/models.log; cat gpurun_out/curve.log | tail -4; tail -3 gpurun_out/prof1.log
find gpurun_out/prof1 -name "*stats*" | head
