#!/bin/bash
# Whole-step knob sweep on the current build (interleaved arms, ROUNDS rounds, bench.py 30 timed steps).
# ARMS: space-separated "name:knob=v,knob=v[:ENV=v,ENV=v]" (knobs via PCMP_KNOBS, then env switches).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
ARMS=${ARMS:-"base: nostream:stream_maxk=0 ewnt:ew_nt=1 epi2:epi_depth=2 nowg8:wgrad8=0"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in $ARMS; do
    IFS=: read -r name k envs <<< "$arm"
    envargs=()
    [ -n "$envs" ] && IFS=, read -r -a envargs <<< "$envs"
    env PCMP_KNOBS="$k" "${envargs[@]}" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-images 0 > gpurun_out/sweep_${name}_$r.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/sweep_${name}_$r.log; exit 1; }
    echo "$name [$k${envs:+ $envs}] $(grep '^{' gpurun_out/sweep_${name}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
