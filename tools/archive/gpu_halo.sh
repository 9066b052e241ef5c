#!/bin/bash
# halo conv kernel: tests, per-shape A/B (knob halo: 0 off, 1 FWD, 3 FWD+DGRAD), then bench off/on
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "halo" > gpurun_out/halo_tests.log 2>&1 || { echo "halo tests failed"; tail -40 gpurun_out/halo_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/halo_tests.log | tail -n 3
timeout -k 10 300 python -u tools/gemm_knob_ab.py --variants 'igemm:halo=0;halo:halo=1;halo_dovl:halo=5' --only l1_3x3,stem --modes fwd,dgrad > gpurun_out/halo_ab.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/halo_ab.log; exit 1; }
grep -v amdgpu gpurun_out/halo_ab.log
for r in 1 2; do
for v in 0 1; do
PCMP_KNOBS="halo=$v" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_h$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_h$v.log; exit 1; }
echo "halo=$v $(grep -o '"value": [0-9.]*' gpurun_out/bench_h$v.log)"
done
done
