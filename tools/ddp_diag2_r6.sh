set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r6_rccl_steps.txt; : > $O
for v in "plain:" "force:--ddp-force" "force-timing:--ddp-force --timing"; do
  n=${v%%:*}; a=${v#*:}
  echo "== $n" >> $O
  timeout -k 10 300 python -u tools/ddp_step_times.py $a --steps 24 --warmup 8 --infer-images 0 >> $O 2>&1 || { echo "$n failed"; tail -20 $O; exit 1; }
  tail -3 $O
done
