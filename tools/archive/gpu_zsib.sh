#!/bin/bash
# 1x1 stride-2 DGRAD sibling-zero epilogue: tests + whole-step A/B (zsib=0: zero fill + accumulate).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sibling or dgrad or conv" > gpurun_out/zsib_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/zsib_tests.log; exit 1; }
tail -1 gpurun_out/zsib_tests.log
for r in 1 2; do
  for v in 0 1; do
    PCMP_KNOBS="zsib=$v" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-images 0 > gpurun_out/zsib_bench_${v}_$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/zsib_bench_${v}_$r.log; exit 1; }
    echo "zsib=$v $(grep '^{' gpurun_out/zsib_bench_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
