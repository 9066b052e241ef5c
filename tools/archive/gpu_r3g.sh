#!/bin/bash
# Coalesced epilogue (epi_coal): kernel tests, conv-shape A/B, whole-step A/B on the new defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3g_tests.log; exit 1; }
tail -2 gpurun_out/r3g_tests.log
timeout -k 10 400 python -u tools/gemm_knob_ab.py --variants 'frag:epi_coal=0;coal:epi_coal=1' --modes fwd,dgrad --rounds 3 > gpurun_out/r3g_shape_ab.txt 2>&1 || { echo knob failed; tail -20 gpurun_out/r3g_shape_ab.txt; exit 1; }
cat gpurun_out/r3g_shape_ab.txt
out=gpurun_out/r3g_ab.txt; : > $out
for r in 1 2 3; do
  for v in 0 1; do
    PCMP_KNOBS=epi_coal=$v timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3g_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3g_b.log; exit 1; }
    echo "round $r coal=$v $(tail -1 gpurun_out/r3g_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
