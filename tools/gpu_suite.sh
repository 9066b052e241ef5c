#!/bin/bash
# Secondary benchmark suite (tools/bench_suite.py, all workloads) -> gpurun_out/suite.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/bench_suite.py $SUITE > gpurun_out/suite.log 2>&1 || { echo "suite failed"; tail -20 gpurun_out/suite.log; exit 1; }
grep '^{' gpurun_out/suite.log
