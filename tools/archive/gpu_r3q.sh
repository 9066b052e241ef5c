#!/bin/bash
# bnr2_n64 knob: BNR2 kernel tests + whole-step A/B; round-3 suite + flagship bench + rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PCMP_KNOBS=bnr2_n64=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bnr2 or fold or dgrad" > gpurun_out/r3q_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3q_tests.log; exit 1; }
tail -1 gpurun_out/r3q_tests.log
out=gpurun_out/r3q_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_KNOBS=bnr2_n64=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3q_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3q_b.log; exit 1; }
    echo "round $r bnr2_n64=$v $(tail -1 gpurun_out/r3q_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
timeout -k 10 900 python -u tools/bench_suite.py > gpurun_out/r3q_suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/r3q_suite.log; exit 1; }
grep '^{' gpurun_out/r3q_suite.log
