#!/bin/bash
# fused BN finalize: kernel tests, then bench with the knob off / on (interleaved, two rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn_" > gpurun_out/kt.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/kt.log; exit 1; }
tail -n 1 gpurun_out/kt.log
for r in 1 2; do
for v in 0 1; do
PCMP_KNOBS="bn_fused_fin=$v" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_ff$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ff$v.log; exit 1; }
echo "bn_fused_fin=$v $(grep -o '"value": [0-9.]*' gpurun_out/bench_ff$v.log)"
done
done
