# forced-RCCL slowdown diagnosis (round 6): kernel trace + stream report of the forced path, then env variants
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_rccl -o run -- \
  python bench.py --ddp-force --opt-after-join --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_rccl.log 2>&1 || { tail -20 gpurun_out/prof_rccl.log; exit 1; }
python tools/stream_report.py gpurun_out/prof_rccl --steps 4 --gaps 25 > gpurun_out/r6_rccl_streams.txt 2>&1
python tools/prof_summary.py gpurun_out/prof_rccl --top 25 --last-steps 4 > gpurun_out/r6_rccl_prof.txt 2>&1
find gpurun_out/prof_rccl -name "*kernel_trace.csv" -delete
head -40 gpurun_out/r6_rccl_streams.txt
: > gpurun_out/r6_rccl_env.txt
for v in "plain:" "force:--ddp-force" "force-q16:--ddp-force PCMP_HW_QUEUES=16" "force-noprio:--ddp-force TORCH_NCCL_HIGH_PRIORITY=0" "force-stepprio0:--ddp-force PCMP_STEP_PRIO=0"; do
  n=${v%%:*}; a=${v#*:}; envs=""; flags=""
  for t in $a; do case $t in --*) flags="$flags $t";; *) envs="$envs $t";; esac; done
  line=$(env $envs timeout -k 10 300 python -u bench.py $flags --steps 20 --warmup 8 --infer-images 0 2>/dev/null | tail -1) || { echo "bench $n failed"; exit 1; }
  echo "$n $line" >> gpurun_out/r6_rccl_env.txt
  echo "$n $line" | cut -c1-140
done
