#!/bin/bash
# Round-end style verification on one GPU: full GPU test suite, smoke(), flagship bench (N=1 defaults).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4v_tests.log 2>&1 || { tail -40 gpurun_out/r4v_tests.log; exit 1; }
tail -2 gpurun_out/r4v_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v_smoke.log 2>&1 || { tail -20 gpurun_out/r4v_smoke.log; exit 1; }
tail -1 gpurun_out/r4v_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4v_bench.txt 2>&1 || { tail -20 gpurun_out/r4v_bench.txt; exit 1; }
tail -1 gpurun_out/r4v_bench.txt | cut -c1-250
