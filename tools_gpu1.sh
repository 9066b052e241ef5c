#!/bin/bash
# first GPU session: kernel numerics, smoke, bench hip vs torch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/kern.log 2>&1; echo "kern rc=$?" >> gpurun_out/kern.log
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log | tail -20; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_hip.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_hip.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --impl torch > gpurun_out/bench_torch.log 2>&1 || { echo torch bench failed; tail -30 gpurun_out/bench_torch.log; }
tail -3 gpurun_out/kern.log; tail -2 gpurun_out/smoke.log; tail -1 gpurun_out/bench_hip.log; tail -1 gpurun_out/bench_torch.log
