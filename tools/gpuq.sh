#!/bin/bash
# Queue one gpurun call: retries ONLY while gpurun answers "no box / slot free" (exit 3, nothing ran,
# nothing charged), up to 40 times 60 s apart.  Any other outcome (including a failed or timed-out
# GPU command) is returned as is: a failing GPU step is never re-run.
# Usage: tools/gpuq.sh <timeout-s> '<command>'   (log: /tmp/gpuq_last.log)
t=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > /tmp/gpuq_last.log 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then tail -4 /tmp/gpuq_last.log; exit $rc; fi
  sleep 60
done
echo "gpuq: no box after 40 tries"; exit 3
