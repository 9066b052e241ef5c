#!/bin/bash
# A/B the 8-wave kernel tile-count threshold: default (240) vs PCMP_IGEMM8_MINTILES=0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 240 0; do
  PCMP_IGEMM8_MINTILES=$v timeout -k 10 200 python tools/conv_micro.py --modes ${MODES:-fwd,dgrad,dgrad_bnr} --only ${ONLY:-l} > gpurun_out/mt_$v.log 2>&1 || { echo "micro $v failed"; tail -5 gpurun_out/mt_$v.log; exit 1; }
done
python - <<'PY'
import json
L = {v: {(r["shape"], r["mode"]): r["us"] for r in map(json.loads, [l for l in open(f"gpurun_out/mt_{v}.log") if l.startswith("{")])} for v in ("240", "0")}
for k in L["240"]:
    print(f"{k[0]:20s} {k[1]:10s} thr240 {L['240'][k]:8.1f}  thr0 {L['0'][k]:8.1f}")
PY
