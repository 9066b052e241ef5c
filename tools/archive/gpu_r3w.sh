#!/bin/bash
# env-knob sweeps on the round-3 build: dz-fold row minimum (layer 1 vs layers 1-2), side-stream WGRAD split target
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r3w_sweep.txt; : > $out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3w_b.log 2>&1 || { echo "bench $label failed"; tail -20 gpurun_out/r3w_b.log; exit 1; }
  echo "$label $(tail -1 gpurun_out/r3w_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
}
for r in 1 2 3; do
  run "r$r minrows=400k" PCMP_DZ_FOLD_MINROWS=400000
  run "r$r minrows=150k" PCMP_DZ_FOLD_MINROWS=150000
  run "r$r side_wgs=256" PCMP_SIDE_WGRAD_WGS=256
  run "r$r side_wgs=512" PCMP_SIDE_WGRAD_WGS=512
done
bash tools/gpu_prof_infer.sh > gpurun_out/r3w_infer_prof.txt 2>&1 || { echo infer prof failed; tail -20 gpurun_out/r3w_infer_prof.txt; exit 1; }
grep -E "p50|per inference" gpurun_out/r3w_infer_prof.txt
find gpurun_out/prof_inf -name "*kernel_trace.csv" -delete; true
