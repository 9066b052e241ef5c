#!/bin/bash
# Round-3 start: plain-GEMM efficiency vs hipBLASLt, per-shape conv kernel table, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/gemm_probe.py --rounds 3 > gpurun_out/r3_gemm_probe.txt 2>&1 || { echo probe failed; tail -20 gpurun_out/r3_gemm_probe.txt; exit 1; }
cat gpurun_out/r3_gemm_probe.txt
timeout -k 10 300 python -u tools/gemm_knob_ab.py --variants 'base:' --rounds 2 > gpurun_out/r3_shape_table.txt 2>&1 || { echo knob failed; tail -20 gpurun_out/r3_shape_table.txt; exit 1; }
cat gpurun_out/r3_shape_table.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_start.log 2>&1 || { echo bench failed; tail -20 gpurun_out/r3_bench_start.log; exit 1; }
tail -1 gpurun_out/r3_bench_start.log
