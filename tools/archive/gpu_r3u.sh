#!/bin/bash
# 64x256 folded stem WGRAD: fold tests, bench x3, tail report
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 200 --timeout-method thread -k "fold or stem or wgrad" > gpurun_out/r3u_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3u_tests.log; exit 1; }
tail -1 gpurun_out/r3u_tests.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3u_b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r3u_b.log; exit 1; }
  echo "round $r $(tail -1 gpurun_out/r3u_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a gpurun_out/r3u_ab.txt
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r3u -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_r3u.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_r3u.log; exit 1; }
python tools/tail_report.py gpurun_out/prof_r3u --steps 1 --last 10 > gpurun_out/r3u_tail.txt
python tools/prof_summary.py gpurun_out/prof_r3u --top 70 --last-steps 4 > gpurun_out/prof_r3u_summary.txt
cat gpurun_out/r3u_tail.txt
find gpurun_out/prof_r3u -name "*kernel_trace.csv" -delete; true
