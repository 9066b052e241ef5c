#!/bin/bash
# Caching-allocator A/B: default segments vs expandable segments at B=256, and B=1024 -> gpurun_out/alloc_ab.log
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PCMP_MEMSTATS=1
run() { echo "== $*" >> gpurun_out/alloc_ab.log; timeout -k 10 300 "$@" >> gpurun_out/alloc_ab.log 2>&1; }
run python bench.py --steps 20 --warmup 5 || { tail -20 gpurun_out/alloc_ab.log; exit 1; }
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True run python bench.py --steps 20 --warmup 5 || { tail -20 gpurun_out/alloc_ab.log; exit 1; }
run python bench.py --steps 5 --warmup 3 --batch-size 1024 || { tail -20 gpurun_out/alloc_ab.log; exit 1; }
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True run python bench.py --steps 5 --warmup 3 --batch-size 1024 || { tail -20 gpurun_out/alloc_ab.log; exit 1; }
grep -E '^==|^\{|\[bench\] mem' gpurun_out/alloc_ab.log | cut -c1-220
