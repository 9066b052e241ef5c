#!/bin/bash
# fp32 wave-quantisation split A/B (round 6): conv micro with f32_qsplit against the default plan,
# then the reference-precision TL flow (ResNet-50 fp32, B=64) with each, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; O=gpurun_out/r6q
for q in ${QS:-5} ${QS2:-}; do timeout -k 10 300 python -u tools/f32_conv_micro.py 64 f32_qsplit=$q > ${O}_micro_$q.txt 2>&1 || { tail -20 ${O}_micro_$q.txt; exit 1; }; done
cat ${O}_micro_*.txt
: > ${O}_tl.txt
for r in 1 2; do  # variants: QS list
  for v in 0 ${QS:-5} ${QS2:-}; do
    PCMP_KNOBS="f32_qsplit=$v" PCMP_PHASE_TIMES=1 timeout -k 10 300 python -u pytorch_training_inference.py --models resnet50 \
      --dtype fp32 --synthetic --json ${O}_tl_$v.json > ${O}_tl_${v}_$r.log 2>&1 || { tail -20 ${O}_tl_${v}_$r.log; exit 1; }
    echo "qsplit=$v round$r $(grep -E 'phase times' ${O}_tl_${v}_$r.log | head -2 | cut -c1-250)" | tee -a ${O}_tl.txt
  done
done
