#!/bin/bash
# BNR2 default change: kernel-variant test + whole-step A/B (old default = streaming kernel, depth 4).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bnr2 or bn_group or stream" > gpurun_out/bnr2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/bnr2_tests.log; exit 1; }
tail -1 gpurun_out/bnr2_tests.log
for r in 1 2; do
  for arm in old new; do
    k=""; [ $arm = old ] && k="stream_bnr2=1,epi_depth_bnr2=4"
    PCMP_KNOBS="$k" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-images 0 > gpurun_out/bnr2_bench_${arm}_$r.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bnr2_bench_${arm}_$r.log; exit 1; }
    echo "$arm $(grep '^{' gpurun_out/bnr2_bench_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
