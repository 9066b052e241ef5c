#!/bin/bash
# embedding-LN tests + BERT A/B, non-pcmp kernel report, full GPU suite, driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_bert_emb.sh || exit 1
timeout -k 10 240 python tools/native_ops_report.py bert > gpurun_out/native_ops_bert.txt 2>&1 || { echo "bert report failed"; tail -30 gpurun_out/native_ops_bert.txt; exit 1; }
timeout -k 10 240 python tools/native_ops_report.py resnet50 > gpurun_out/native_ops_resnet50.txt 2>&1 || { echo "resnet report failed"; tail -30 gpurun_out/native_ops_resnet50.txt; exit 1; }
grep -v "amdgpu.ids\|GPU_MAX_HW" gpurun_out/native_ops_bert.txt gpurun_out/native_ops_resnet50.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/combo_pytest_gpu.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/combo_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/combo_pytest_gpu.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/combo_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/combo_bench.log; exit 1; }
tail -1 gpurun_out/combo_bench.log
