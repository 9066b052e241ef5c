#!/bin/bash
# Class-blocked transposed weights for stride-2 DGRAD: tests + whole-step A/B (PCMP_S2_CLASS_T=0: per-call transposes).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s2t_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/s2t_tests.log; exit 1; }
tail -1 gpurun_out/s2t_tests.log
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_S2_CLASS_T=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-images 0 > gpurun_out/s2t_bench_${v}_$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/s2t_bench_${v}_$r.log; exit 1; }
    echo "s2t=$v $(grep '^{' gpurun_out/s2t_bench_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
