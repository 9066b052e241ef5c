#!/bin/bash
# ResNet-50 transfer-learning step (B=64) under kernel/env variants, to locate a regression.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for arm in "base:" "halo0:halo=0" "pool0:pool3s2=0" "q4::PCMP_HW_QUEUES=4" "s2d0::PCMP_STEM_S2D=0"; do
    IFS=: read -r name k envs <<< "$arm"
    envargs=(); [ -n "$envs" ] && IFS=, read -r -a envargs <<< "$envs"
    env PCMP_KNOBS="$k" "${envargs[@]}" timeout -k 10 300 python tools/bench_suite.py resnet50_tl_train > gpurun_out/tl_${name}_$r.log 2>&1 || { echo "tl $name failed"; tail -20 gpurun_out/tl_${name}_$r.log; exit 1; }
    echo "$name $(grep '"impl": "hip"' gpurun_out/tl_${name}_$r.log | cut -c1-120)"
  done
done
