#!/bin/bash
# In-kernel split-K fixup (sk_fixup): kernel tests, then BERT / batch-1 inference / ResNet-50 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_text_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3m_tests.log 2>&1 || { echo tests failed; tail -40 gpurun_out/r3m_tests.log; exit 1; }
tail -2 gpurun_out/r3m_tests.log
out=gpurun_out/r3m_ab.txt; : > $out
for r in 1 2; do
  for v in 0 1; do
    PCMP_KNOBS=sk_fixup=$v,wgrad_dma=0 SUITE_HIP_ONLY=1 timeout -k 10 300 python -u tools/bench_suite.py bert_train resnet50_infer > gpurun_out/r3m_bb.log 2>&1 || { echo "suite $v failed"; tail -20 gpurun_out/r3m_bb.log; exit 1; }
    grep -E "bert_train|resnet50_infer" gpurun_out/r3m_bb.log | sed "s/^/round $r sk_fixup=$v /" | tee -a $out
  done
done
for r in 1 2; do
  for v in 0 1; do
    PCMP_KNOBS=sk_fixup=$v,wgrad_dma=0 timeout -k 10 200 python bench.py --steps 30 --warmup 8 --infer-images 0 > gpurun_out/r3m_b.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/r3m_b.log; exit 1; }
    echo "round $r resnet sk_fixup=$v $(tail -1 gpurun_out/r3m_b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["final_loss"])')" | tee -a $out
  done
done
