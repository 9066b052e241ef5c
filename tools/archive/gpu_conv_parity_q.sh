#!/bin/bash
# ResNet-18 convergence-parity test (pcmp vs torch autocast in one process) at 4 and 8 HW queues.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  for q in 4 8; do
    PCMP_HW_QUEUES=$q timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -q -s --timeout 240 --timeout-method thread -k convergence > gpurun_out/cq_${q}_$r.log 2>&1
    echo "q=$q r=$r rc=$? $(grep 'resnet18 convergence' gpurun_out/cq_${q}_$r.log)"
  done
done
