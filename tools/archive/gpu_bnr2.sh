#!/bin/bash
# Dual BN-reduce DGRAD (EPI_BNR2): persistent streaming kernel (spills 112 B/lane) vs the one-tile kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python tools/gemm_knob_ab.py --modes dgrad --only l1_1x1_256to64,l2_1x1_512to128,l3_1x1_1024to256 --rounds 3 --variants 'stream:;onetile:stream_bnr2=0;onetile_d2:stream_bnr2=0,epi_depth=2' > gpurun_out/bnr2_ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/bnr2_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bnr2_ab.txt
