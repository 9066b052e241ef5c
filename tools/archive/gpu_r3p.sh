#!/bin/bash
# layer-1-only BatchNorm-backward fold: whole-step A/B; then the round-3 serial layer profile
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r3p_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_DZ_FOLD=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3p_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3p_b.log; exit 1; }
    echo "round $r dz_fold=$v $(tail -1 gpurun_out/r3p_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
PCMP_WGRAD_STREAM=0 timeout -k 10 300 python -u tools/layer_profile.py --top 60 > gpurun_out/r3p_layer_profile.txt 2>&1 || { echo layer profile failed; tail -20 gpurun_out/r3p_layer_profile.txt; exit 1; }
head -30 gpurun_out/r3p_layer_profile.txt
