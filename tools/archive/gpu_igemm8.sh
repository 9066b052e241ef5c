#!/bin/bash
# 8-wave kernel validation: numerics on large shapes, then conv microbench with the kernel on/off.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "large_shapes or conv_fwd or conv_dgrad" > gpurun_out/t8.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t8.log; exit 1; }
tail -2 gpurun_out/t8.log
PCMP_IGEMM8=0 timeout -k 10 200 python tools/conv_micro.py --modes fwd,dgrad,dgrad_bnr > gpurun_out/m_old.log 2>&1 || { echo "micro old failed"; tail -5 gpurun_out/m_old.log; exit 1; }
PCMP_IGEMM8=1 timeout -k 10 200 python tools/conv_micro.py --modes fwd,dgrad,dgrad_bnr > gpurun_out/m_new.log 2>&1 || { echo "micro new failed"; tail -5 gpurun_out/m_new.log; exit 1; }
python - <<'PY'
import json
o = {(r["shape"], r["mode"]): r["us"] for r in map(json.loads, [l for l in open("gpurun_out/m_old.log") if l.startswith("{")])}
for l in open("gpurun_out/m_new.log"):
    if l.startswith("{"):
        r = json.loads(l)
        print(f'{r["shape"]:20s} {r["mode"]:10s} old {o[(r["shape"], r["mode"])]:8.1f}  new {r["us"]:8.1f}  tflops {r["tflops"]}')
PY
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench8.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench8.log; exit 1; }
tail -1 gpurun_out/bench8.log
