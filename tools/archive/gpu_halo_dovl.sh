#!/bin/bash
# overlapped BN-backward DGRAD on the halo kernel (knob halo bit 2): per-shape A/B, then bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gemm_knob_ab.py --variants 'igemm:halo=1;halo_dovl:halo=5' --only l1_3x3 --modes dgrad > gpurun_out/halo_dovl_ab.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/halo_dovl_ab.log; exit 1; }
grep -v amdgpu gpurun_out/halo_dovl_ab.log
for r in 1 2; do
for v in 1 5; do
PCMP_KNOBS="halo=$v" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_d$v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_d$v.log; exit 1; }
echo "halo=$v $(grep -o '"value": [0-9.]*' gpurun_out/bench_d$v.log)"
done
done
