#!/bin/bash
# tools/gemm_knob_ab.py on the GPU: VARIANTS / ONLY / MODES from the environment.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ab}
timeout -k 10 500 python -u tools/gemm_knob_ab.py --variants "$VARIANTS" ${ONLY:+--only $ONLY} ${MODES:+--modes $MODES} > gpurun_out/knob_$TAG.log 2>&1 || { echo ab failed; tail -30 gpurun_out/knob_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/knob_$TAG.log
