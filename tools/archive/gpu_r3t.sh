#!/bin/bash
# stem tail mode (PCMP_STEM_TAIL): gradient test, whole-step A/B, tail report of the new default
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3t_tests.log; exit 1; }
tail -1 gpurun_out/r3t_tests.log
out=gpurun_out/r3t_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_STEM_TAIL=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3t_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3t_b.log; exit 1; }
    echo "round $r stem_tail=$v $(tail -1 gpurun_out/r3t_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3t -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_r3t.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_r3t.log; exit 1; }
python tools/tail_report.py gpurun_out/prof_r3t --steps 2 --last 16 > gpurun_out/r3t_tail.txt
cat gpurun_out/r3t_tail.txt
find gpurun_out/prof_r3t -name "*kernel_trace.csv" -delete; true
