#!/bin/bash
# Full GPU test suite + flagship bench (one GPU).  Outputs gpurun_out/r4_full_tests.log, r4_full_bench.txt
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_full_tests.log 2>&1 || { tail -40 gpurun_out/r4_full_tests.log; exit 1; }
tail -3 gpurun_out/r4_full_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4_full_bench.txt 2>&1 || { tail -20 gpurun_out/r4_full_bench.txt; exit 1; }
tail -1 gpurun_out/r4_full_bench.txt
