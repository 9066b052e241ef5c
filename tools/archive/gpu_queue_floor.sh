#!/bin/bash
# The pool exports GPU_MAX_HW_QUEUES=4; pcmp now raises it to 8.  Plain vs forced-RCCL bench under
# torchrun (the driver's launch form), interleaved, with the box's environment untouched.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-<unset>}"
python -c "import pcmp, os; print('after import pcmp:', os.environ['GPU_MAX_HW_QUEUES'])"
for r in 1 2; do
  for arm in plain force; do
    extra=""; [ $arm = force ] && extra="--ddp-force"
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 30 --warmup 5 --infer-images 0 $extra > gpurun_out/qf_${arm}_$r.log 2>&1 || { echo "bench $arm failed"; tail -30 gpurun_out/qf_${arm}_$r.log; exit 1; }
    echo "$arm $r $(grep '^{' gpurun_out/qf_${arm}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["ddp_force"])')"
  done
done
