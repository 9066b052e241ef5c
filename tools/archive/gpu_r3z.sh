#!/bin/bash
# compile-time A/B: default build (epi_coal / bn_group compiled out) vs the variant with them compiled in
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
ALT=$GRAFT_REPO_ROOT/performance-comparison-of-tensorflow-pytorch-and-their-distributed-counterparts_amd/_native/libpcmp_hip_allepi.so
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3z_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3z_tests.log; exit 1; }
tail -1 gpurun_out/r3z_tests.log
out=gpurun_out/r3z_ab.txt; : > $out
for r in 1 2 3; do
  for v in default allepi; do
    if [ $v = allepi ]; then export PCMP_LIB=$ALT; else unset PCMP_LIB; fi
    timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 100 > gpurun_out/r3z_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3z_b.log; exit 1; }
    echo "round $r $v $(tail -1 gpurun_out/r3z_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference_p50_ms"], d["config"]["final_loss"])')" | tee -a $out
  done
done
unset PCMP_LIB
