#!/bin/bash
# Whole-step interleaved A/B of environment switches on the flagship bench (one process per run):
# VARIANTS="name:VAR=v VAR2=v;name2:VAR=v" ROUNDS=3 -> gpurun_out/r4_env_ab.txt
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
out=gpurun_out/r4_env_ab.txt
: > $out
IFS=';' read -ra VS <<< "$VARIANTS"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "${VS[@]}"; do
    name=${v%%:*}; envs=${v#*:}
    line=$(env $envs timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-8} --infer-images 0 2>/dev/null | tail -1) || { echo "bench $name failed"; exit 1; }
    echo "$name round$r $line" | tee -a $out | cut -c1-180
  done
done
