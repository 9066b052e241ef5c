#!/bin/bash
# Whole-step interleaved A/B of kernel knobs on the flagship bench (one process per run, same box):
# VARIANTS="name=knobs;name=knobs" ROUNDS=3 -> gpurun_out/r4_bench_ab.txt (one JSON line per run)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r4_bench_ab.txt
: > $out
IFS=';' read -ra VS <<< "${VARIANTS:-base=big=0;big=big=3}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in "${VS[@]}"; do
    name=${v%%=*}; knobs=${v#*=}
    line=$(PCMP_KNOBS="$knobs" timeout -k 10 240 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-8} \
           --infer-images 0 2>/dev/null | tail -1) || { echo "bench $name failed"; exit 1; }
    echo "$name round$r $line" | tee -a $out | cut -c1-200
  done
done
