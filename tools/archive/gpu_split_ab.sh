#!/bin/bash
# Batch-1 inference split-K A/B: PCMP_FWD_SPLIT_TARGET x PCMP_FWD_SPLIT_MINK -> gpurun_out/split_ab.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/split_ab.log
if [ -n "$CFG_LIST" ]; then IFS=, read -ra CFGS <<< "$CFG_LIST"; else CFGS=("256 4" "128 4" "512 4" "256 8" "128 8" "64 8" "256 4"); fi
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  echo "== target $1 mink $2" >> $L
  PCMP_FWD_SPLIT_TARGET=$1 PCMP_FWD_SPLIT_MINK=$2 timeout -k 10 200 python tools/bench_suite.py resnet50_infer >> $L 2>&1 || { tail -20 $L; exit 1; }
done
grep -E '^==|hip\+graph' $L | cut -c1-120
