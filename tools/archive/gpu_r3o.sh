#!/bin/bash
# per-shape cost of the BatchNorm-backward fold (tools/fold_micro.py)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/fold_micro.py --rounds 3 > gpurun_out/r3o_fold_micro.txt 2>&1 || { echo micro failed; tail -30 gpurun_out/r3o_fold_micro.txt; exit 1; }
cat gpurun_out/r3o_fold_micro.txt
