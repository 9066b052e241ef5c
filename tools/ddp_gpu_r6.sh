# round 6: forced-RCCL (one GPU, world 1) headline-config bench records: per-bucket optimizer vs
# one update after the join, fp32 / bf16 gradient all-reduce; the plain step interleaved as control
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r6_rccl_force.txt; : > $O
for r in 1 2 3; do
for v in "plain:" "perbucket-fp32:--ddp-force" "afterjoin-fp32:--ddp-force --opt-after-join" "perbucket-bf16:--ddp-force --grad-dtype bf16"; do
  n=${v%%:*}; a=${v#*:}
  line=$(timeout -k 10 300 python -u bench.py --batch-size 256 --steps 20 --warmup 8 --infer-images 0 $a 2>/dev/null | tail -1) || { echo "bench $n failed"; exit 1; }
  echo "$n round$r $line" >> $O
  echo "$n round$r $line" | cut -c1-150
done; done
