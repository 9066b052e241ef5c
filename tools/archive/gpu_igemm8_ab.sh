#!/bin/bash
# A/B the 8-wave kernel: PCMP_IGEMM8=0 (4-wave kernel), 1 (8-wave), 2 (8-wave + MFMA priority)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 1 2; do
  PCMP_IGEMM8=$v timeout -k 10 200 python tools/conv_micro.py --modes ${MODES:-fwd,dgrad,dgrad_bnr} > gpurun_out/m_$v.log 2>&1 || { echo "micro $v failed"; tail -5 gpurun_out/m_$v.log; exit 1; }
done
python - <<'PY'
import json
L = {v: {(r["shape"], r["mode"]): r["us"] for r in map(json.loads, [l for l in open(f"gpurun_out/m_{v}.log") if l.startswith("{")])} for v in "012"}
for k in L["0"]:
    print(f"{k[0]:20s} {k[1]:10s} 4w {L['0'][k]:8.1f}  8w {L['1'][k]:8.1f}  8w+prio {L['2'][k]:8.1f}")
PY
