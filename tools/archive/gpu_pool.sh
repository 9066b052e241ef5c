#!/bin/bash
# Stem pooling kernels: correctness tests, in-process A/B, flagship bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or maxpool or stem" > gpurun_out/pool_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pool_tests.log; exit 1; }
tail -2 gpurun_out/pool_tests.log
timeout -k 10 200 python tools/pool_ab.py > gpurun_out/pool_ab.txt 2>&1 || { echo "pool ab failed"; tail -20 gpurun_out/pool_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/pool_ab.txt
for r in 1 2; do
  for v in 0 1; do
    PCMP_KNOBS="pool3s2=$v" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-images 0 > gpurun_out/pool_bench_${v}_$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/pool_bench_${v}_$r.log; exit 1; }
    echo "pool3s2=$v $(grep '^{' gpurun_out/pool_bench_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
