#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -q -m gpu -x > gpurun_out/eng.log 2>&1; echo "eng rc=$?" >> gpurun_out/eng.log
timeout -k 10 600 python tools/bench_suite.py > gpurun_out/suite.log 2>&1; echo "suite rc=$?" >> gpurun_out/suite.log
tail -5 gpurun_out/eng.log; cat gpurun_out/suite.log | grep -v Warn | tail -20
