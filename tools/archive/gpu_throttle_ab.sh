#!/bin/bash
# Host run-ahead throttle A/B (PCMP_MAX_INFLIGHT=0 = unbounded) at B=256 and B=1024, plus the
# throttle / engine GPU tests -> gpurun_out/throttle_ab.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PCMP_MEMSTATS=1
L=gpurun_out/throttle_ab.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "throttle or tl_flow" >> $L 2>&1 || { tail -30 $L; exit 1; }
run() { echo "== $*" >> $L; timeout -k 10 300 "$@" >> $L 2>&1; }
PCMP_MAX_INFLIGHT=0 run python bench.py --steps 20 --warmup 5 || { tail -20 $L; exit 1; }
run python bench.py --steps 20 --warmup 5 || { tail -20 $L; exit 1; }
PCMP_MAX_INFLIGHT=1 run python bench.py --steps 20 --warmup 5 || { tail -20 $L; exit 1; }
run python bench.py --steps 5 --warmup 3 --batch-size 1024 || { tail -20 $L; exit 1; }
run python bench.py --steps 20 --warmup 5 --model resnet18 || { tail -20 $L; exit 1; }
grep -E 'passed|failed|^==|^\{|\[bench\] mem' $L | cut -c1-200
