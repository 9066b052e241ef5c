#!/bin/bash
# A/B an env switch on the conv microbench: VAR=<name> A=<val> B=<val> [ONLY=<shape substr>] [MODES=...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "$A" "$B"; do
  env $VAR=$v timeout -k 10 200 python tools/conv_micro.py --modes ${MODES:-fwd,dgrad,dgrad_bnr} --only ${ONLY:-_} > gpurun_out/ab_$v.log 2>&1 || { echo "micro $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
done
python - "$A" "$B" <<'PY'
import json, sys
a, b = sys.argv[1], sys.argv[2]
L = {v: {(r["shape"], r["mode"]): r["us"] for r in map(json.loads, [l for l in open(f"gpurun_out/ab_{v}.log") if l.startswith("{")])} for v in (a, b)}
for k in L[a]:
    print(f"{k[0]:20s} {k[1]:10s} {a}: {L[a][k]:8.1f}  {b}: {L[b][k]:8.1f}")
PY
