#!/bin/bash
# Side-stream WGRAD split target (PCMP_SIDE_WGRAD_WGS, default 384) vs per-shape autotune (0): model tests + whole-step A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_model_parity_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/sw_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/sw_tests.log; exit 1; }
tail -1 gpurun_out/sw_tests.log
for r in 1 2 3; do
  for v in 0 384; do
    PCMP_SIDE_WGRAD_WGS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-images 0 > gpurun_out/sw_bench_${v}_$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/sw_bench_${v}_$r.log; exit 1; }
    echo "side_wgs=$v $(grep '^{' gpurun_out/sw_bench_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
