#!/bin/bash
# batch-1 inference latency with the small-M plan off / on (same process order: off first), kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/kt.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
timeout -k 10 300 python -u tools/infer_plan_ab.py > gpurun_out/infer_ab.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/infer_ab.log; exit 1; }
grep -v amdgpu gpurun_out/infer_ab.log
