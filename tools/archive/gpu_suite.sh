#!/bin/bash
# secondary benchmark suite (ResNet-18, ResNet-50 TL, batch-1 inference, BiLSTM, BERT) + flagship bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_suite.py > gpurun_out/suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/suite.log; exit 1; }
grep '^{' gpurun_out/suite.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
grep metric gpurun_out/bench.log
