#!/bin/bash
# non-pcmp kernels of one BERT-base and one ResNet-50 training step, with the issuing source line
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/native_ops_report.py bert > gpurun_out/native_ops_bert.txt 2>&1 || { echo "bert failed"; tail -30 gpurun_out/native_ops_bert.txt; exit 1; }
timeout -k 10 300 python tools/native_ops_report.py resnet50 > gpurun_out/native_ops_resnet50.txt 2>&1 || { echo "resnet failed"; tail -30 gpurun_out/native_ops_resnet50.txt; exit 1; }
grep -v "amdgpu.ids\|GPU_MAX_HW" gpurun_out/native_ops_bert.txt gpurun_out/native_ops_resnet50.txt
