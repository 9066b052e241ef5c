#!/bin/bash
# RCCL forced-collective path on one GPU: GPU tests, bench A/B (plain vs --ddp-force fp32 / bf16),
# and a rocprofv3 kernel trace of the forced run (RCCL kernels next to backward kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ddp_rccl_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ddp_rccl_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/ddp_rccl_tests.log; exit 1; }
tail -5 gpurun_out/ddp_rccl_tests.log
run() {  # $1 = label, rest = bench args
  local lab=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=$((29500 + RANDOM % 1000)) bench.py --gpus 1 --steps 30 --warmup 5 "$@" > gpurun_out/ddpf_$lab.log 2>&1 || { echo "bench $lab failed"; tail -30 gpurun_out/ddpf_$lab.log; exit 1; }
  echo "$lab $(grep '^{' gpurun_out/ddpf_$lab.log)"
}
for r in 1 2; do
  run plain_$r || exit 1
  run force_fp32_$r --ddp-force || exit 1
  run force_bf16_$r --ddp-force --grad-dtype bf16 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ddpf -o run -- python bench.py --steps 5 --warmup 2 --ddp-force --infer-images 0 > gpurun_out/prof_ddpf.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_ddpf.log; exit 1; }
echo profiled
