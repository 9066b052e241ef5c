#!/bin/bash
# ResNet-18 convergence-parity test, three runs (reference stability check).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -q -s --timeout 240 --timeout-method thread -k convergence > gpurun_out/cp_$r.log 2>&1
  echo "r=$r rc=$? $(grep 'resnet18 convergence' gpurun_out/cp_$r.log | tail -1)"
done
