#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/grad_diag.py > gpurun_out/graddiag.log 2>&1
ARCH=resnet18 timeout -k 10 300 python tools/grad_diag.py > gpurun_out/graddiag18.log 2>&1
tail -4 gpurun_out/graddiag.log; tail -4 gpurun_out/graddiag18.log
