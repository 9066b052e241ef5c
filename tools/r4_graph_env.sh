#!/bin/bash
# BERT whole-step hipGraph (with the WGRAD side stream) under HIP runtime graph settings, one process
# per setting: does the runtime's graph-branch queue assignment explain the slow multi-stream replay?
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
out=gpurun_out/r4_graph_env.txt; : > $out
for cfg in "default:" "gq1:DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "gq2:DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "gq4:DEBUG_HIP_FORCE_GRAPH_QUEUES=4" \
           "pc0:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "pc1:DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
  name=${cfg%%:*}; kv=${cfg#*:}
  echo "== $name $kv" >> $out
  if [ -n "$kv" ]; then export "$kv"; fi
  timeout -k 10 240 python -u tools/bert_ab.py --variants "side:;graph:GRAPH=1" --rounds 2 --steps 30 2>&1 | grep round >> $out || { echo "$name failed" >> $out; exit 1; }
  if [ -n "$kv" ]; then unset "${kv%%=*}"; fi
done
cat $out
