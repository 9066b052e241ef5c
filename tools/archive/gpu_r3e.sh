#!/bin/bash
# Full GPU test suite (fp32 path, new loss kernels, PF2 fix) + smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_f32_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3e_f32.log 2>&1 || { echo f32 tests failed; tail -40 gpurun_out/r3e_f32.log; exit 1; }
tail -3 gpurun_out/r3e_f32.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e_pytest_gpu.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3e_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r3e_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3e_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r3e_smoke.log; exit 1; }
tail -1 gpurun_out/r3e_smoke.log
