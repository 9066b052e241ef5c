#!/bin/bash
# End-of-session verification on the committed build: full GPU test suite, smoke, the driver's
# bench command (N=1), the forced RCCL path under torchrun, and a steady-state rocprofv3 kernel table.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/final_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --steps 20 --warmup 5 --infer-images 0 --ddp-force > gpurun_out/final_bench_ddp.log 2>&1 || { echo "ddp bench failed"; tail -20 gpurun_out/final_bench_ddp.log; exit 1; }
grep '^{' gpurun_out/final_bench_ddp.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_final.log 2>&1 || { echo rocprof failed; tail -30 gpurun_out/prof_final.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_final --top 60 --last-steps 4 > gpurun_out/prof_final_summary.txt
sed -n '/per step over/,$p' gpurun_out/prof_final_summary.txt | head -12
find gpurun_out/prof_final -name "*kernel_trace.csv" -delete
