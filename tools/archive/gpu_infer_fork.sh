#!/bin/bash
# batch-1 inference: eval downsample fork off/on, then the inference + model tests
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/infer_fork_ab.py > gpurun_out/infer_fork.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/infer_fork.log; exit 1; }
grep -v amdgpu gpurun_out/infer_fork.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "infer or batch1 or eval or parity" > gpurun_out/kt.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/kt.log; exit 1; }
tail -n 1 gpurun_out/kt.log
