#!/bin/bash
# One entry point for the GPU-box work (replaces round 4's per-experiment tools/r4_*.sh wrappers).
#
#   gpurun -- bash tools/gpu.sh TASK [TASK ...]
#
# Tasks run in order; the first failure ends the call (no GPU step after a failed one).  Every
# output goes to gpurun_out/${TAG}_<task>.* (TAG defaults to r5).  Each GPU step has its own time
# limit.  Tasks:
#   tests        pytest -m gpu over ${TESTS:-tests} (optional -k "$K")
#   verify       full GPU test suite + smoke() + flagship bench (the driver's round-end sequence)
#   bench        flagship bench, N=1 defaults
#   bench-ab     interleaved whole-step knob A/B: VARIANTS="name=k=v,k=v;name2=..." ROUNDS STEPS WARMUP
#   env-ab       interleaved whole-step environment A/B: VARIANTS="name:VAR=v VAR2=v;name2:..."
#   knob-ab      per-shape in-process knob A/B (tools/gemm_knob_ab.py): KVARIANTS='a:k=v;b:k=v' MODES
#   prof-bench   rocprofv3 kernel stats + per-step table of the ResNet-50 bench step
#   prof-bert    rocprofv3 kernel stats + per-step table of the BERT-base step
#   prof-r18     rocprofv3 kernel stats + stream report of the ResNet-18 B=256 training step
#   prof-bilstm  rocprofv3 kernel stats + per-step table of the BiLSTM step (B=32, S=128)
#   prof-infer   rocprofv3 trace of the batch-1 hipGraph inference loop: kernels / span per image
#   tail         end-of-backward tail report (tools/tail_report.py)
#   layer        serial event-bracketed layer profile (WGRAD side stream off)
#   suite        secondary workloads (tools/bench_suite.py, HIP only)
#   bert         BERT text-path tests, GEMM / attention micro benchmarks, whole-step A/B (BVARIANTS)
#   pmc-dgrad    PMC passes over the isolated layer-1 DGRAD + BN-reduce shape
#   prof-f32     rocprofv3 kernel stats of the fp32 transfer-learning forward (B=64)
#   f32          fp32 conv micro (tools/f32_conv_micro.py) + the reference-precision ResNet-50 rerun
#                (pytorch_training_inference.py --dtype fp32: TL forward ms/step, batch-1 p50)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r6}
O=gpurun_out/$T

die() { echo "[$1 failed]"; [ -n "$2" ] && tail -40 "$2"; exit 1; }

task_tests() {
  local kk=(); [ -n "$K" ] && kk=(-k "$K")
  timeout -k 10 ${TIMEOUT:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread \
    "${kk[@]}" > ${O}_tests.log 2>&1 || die tests ${O}_tests.log
  tail -2 ${O}_tests.log
}
task_bench() {
  timeout -k 10 300 python -u bench.py > ${O}_bench.txt 2>&1 || die bench ${O}_bench.txt
  tail -1 ${O}_bench.txt | cut -c1-300
}
task_verify() {
  TESTS=tests K= task_tests
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 || die smoke ${O}_smoke.log
  tail -1 ${O}_smoke.log
  task_bench
}
task_bench_ab() {
  local out=${O}_bench_ab.txt; : > $out
  IFS=';' read -ra VS <<< "$VARIANTS"
  for r in $(seq 1 ${ROUNDS:-3}); do
    for v in "${VS[@]}"; do
      local name=${v%%=*} knobs=${v#*=}
      local line
      line=$(PCMP_KNOBS="$knobs" timeout -k 10 240 python -u bench.py ${BENCH_ARGS:-} --steps ${STEPS:-20} --warmup ${WARMUP:-8} \
             --infer-images ${INFER:-0} 2>/dev/null | tail -1) || die "bench-ab $name"
      echo "$name round$r $line" | tee -a $out | cut -c1-200
    done
  done
}
task_env_ab() {
  local out=${O}_env_ab.txt; : > $out
  IFS=';' read -ra VS <<< "$VARIANTS"
  for r in $(seq 1 ${ROUNDS:-3}); do
    for v in "${VS[@]}"; do
      local name=${v%%:*} envs=${v#*:}
      local line
      line=$(env $envs timeout -k 10 240 python -u bench.py ${BENCH_ARGS:-} --steps ${STEPS:-20} --warmup ${WARMUP:-8} \
             --infer-images ${INFER:-0} 2>/dev/null | tail -1) || die "env-ab $name"
      echo "$name round$r $line" | tee -a $out | cut -c1-200
    done
  done
}
task_knob_ab() {
  timeout -k 10 600 python -u tools/gemm_knob_ab.py --variants "$KVARIANTS" --modes ${MODES:-fwd,dgrad,wgrad} \
    --rounds ${ROUNDS:-3} ${ONLY:+--only $ONLY} > ${O}_knob_ab.txt 2>&1 || die knob-ab ${O}_knob_ab.txt
  cat ${O}_knob_ab.txt
}
task_prof_bench() {
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
    python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_bench.log 2>&1 || die prof-bench gpurun_out/prof_bench.log
  python tools/prof_summary.py gpurun_out/prof_bench --top 60 --last-steps 4 > ${O}_prof_bench.txt
  python tools/stream_report.py gpurun_out/prof_bench --steps 4 > ${O}_streams.txt 2>&1
  find gpurun_out/prof_bench -name "*kernel_trace.csv" -delete
  head -12 ${O}_streams.txt
  sed -n '/per step over/,+12p' ${O}_prof_bench.txt
}
task_prof_bert() {
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bert -o run -- \
    python tools/prof_target.py bert 16 > gpurun_out/prof_bert.log 2>&1 || die prof-bert gpurun_out/prof_bert.log
  python tools/prof_summary.py gpurun_out/prof_bert --top 45 --step-kernel adam_flat --last-steps 4 > ${O}_prof_bert.txt
  python tools/stream_report.py gpurun_out/prof_bert --steps 4 --step-kernel adam_flat --loss-kernel xent --gaps 30 \
    > ${O}_bert_streams.txt 2>&1 || true
  find gpurun_out/prof_bert -name "*kernel_trace.csv" -delete
  sed -n '/per step over/,+12p' ${O}_prof_bert.txt
}
task_prof_bilstm() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bilstm -o run -- \
    python tools/prof_target.py bilstm 16 > gpurun_out/prof_bilstm.log 2>&1 || die prof-bilstm gpurun_out/prof_bilstm.log
  python tools/prof_summary.py gpurun_out/prof_bilstm --top 30 --step-kernel adam_flat --last-steps 4 > ${O}_prof_bilstm.txt
  find gpurun_out/prof_bilstm -name "*kernel_trace.csv" -delete
  sed -n '/per step over/,+12p' ${O}_prof_bilstm.txt
}
task_prof_r18() {   # ResNet-18 B=256 training step (BASELINE.json config 2): kernel stats + stream report
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r18 -o run -- \
    python tools/prof_target.py resnet18 12 > gpurun_out/prof_r18.log 2>&1 || die prof-r18 gpurun_out/prof_r18.log
  python tools/prof_summary.py gpurun_out/prof_r18 --top 40 --last-steps 4 > ${O}_prof_r18.txt
  python tools/stream_report.py gpurun_out/prof_r18 --steps 4 > ${O}_r18_streams.txt 2>&1 || true
  find gpurun_out/prof_r18 -name "*kernel_trace.csv" -delete
  head -8 ${O}_r18_streams.txt
  sed -n '/per step over/,+30p' ${O}_prof_r18.txt
}
task_prof_f32() {   # fp32 transfer-learning forward (B=64): kernel stats over 10 forwards
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_f32 -o run -- \
    python $R/tools/prof_target.py resnet50_f32_tl 10 > $R/gpurun_out/prof_f32.log 2>&1 || die prof-f32 $R/gpurun_out/prof_f32.log
  cd $R
  python tools/prof_summary.py gpurun_out/prof_f32 --top 40 --steps 10 --last-steps 0 > ${O}_prof_f32.txt
  find gpurun_out/prof_f32 -name "*kernel_trace.csv" -delete
  head -50 ${O}_prof_f32.txt
}
task_prof_infer() {
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inf -o run -- \
    python tools/prof_infer.py 200 > gpurun_out/prof_inf.log 2>&1 || die prof-infer gpurun_out/prof_inf.log
  grep p50 gpurun_out/prof_inf.log
  python tools/prof_summary.py gpurun_out/prof_inf --top 30 --last-steps 0 > ${O}_prof_infer.txt
  python tools/infer_timeline.py gpurun_out/prof_inf >> ${O}_prof_infer.txt
  find gpurun_out/prof_inf -name "*kernel_trace.csv" -delete
  grep "per inference" ${O}_prof_infer.txt
}
task_tail() {
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tail -o run -- \
    python bench.py --steps 6 --warmup 3 --infer-images 0 > gpurun_out/prof_tail.log 2>&1 || die tail gpurun_out/prof_tail.log
  python tools/tail_report.py gpurun_out/prof_tail --steps 3 --last 24 > ${O}_tail.txt 2>&1
  find gpurun_out/prof_tail -name "*kernel_trace.csv" -delete
  head -40 ${O}_tail.txt
}
task_layer() {
  PCMP_WGRAD_STREAM=0 timeout -k 10 300 python tools/layer_profile.py --top 60 > ${O}_layer_profile.txt 2>&1 || die layer ${O}_layer_profile.txt
  head -30 ${O}_layer_profile.txt
}
task_suite() {
  SUITE_HIP_ONLY=${SUITE_HIP_ONLY:-1} timeout -k 10 600 python -u tools/bench_suite.py > ${O}_bench_suite.txt 2>&1 || die suite ${O}_bench_suite.txt
  grep "^{" ${O}_bench_suite.txt | cut -c1-200
}
task_bert() {
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_text_f32_gpu.py \
    tests/test_text_kernels_gpu.py > ${O}_bert_tests.log 2>&1 || die bert-tests ${O}_bert_tests.log
  tail -2 ${O}_bert_tests.log
  timeout -k 10 300 python -u tools/bert_gemm_micro.py --rounds 3 > ${O}_bert_gemm_micro.txt 2>&1 || die bert-gemm
  timeout -k 10 200 python -u tools/attn_micro.py > ${O}_attn_micro.txt 2>&1 || die attn-micro
  timeout -k 10 600 python -u tools/bert_ab.py --variants "${BVARIANTS:-serial:PCMP_WGRAD_STREAM=0;side:}" --rounds 3 \
    > ${O}_bert_ab.txt 2>&1 || die bert-ab ${O}_bert_ab.txt
  cat ${O}_bert_ab.txt
}
task_pmc_dgrad() {
  mkdir -p $R/gpurun_out/pmc; cd /tmp
  timeout -k 10 120 python -u $R/tools/dgrad_pmc.py > $R/gpurun_out/pmc/time.txt 2>&1 || die pmc-time
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/pmc/p1 -o run -- \
    python $R/tools/dgrad_pmc.py > $R/gpurun_out/pmc/p1.log 2>&1 || die pmc-p1 $R/gpurun_out/pmc/p1.log
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv \
    -d $R/gpurun_out/pmc/p2 -o run -- python $R/tools/dgrad_pmc.py > $R/gpurun_out/pmc/p2.log 2>&1 || die pmc-p2 $R/gpurun_out/pmc/p2.log
  cd $R
}
task_pmc_wgrad() {   # SHAPE=l3_3x3 ...: three passes (LDS, waits / MFMA, memory) over tools/wgrad_pmc.py
  mkdir -p $R/gpurun_out/pmcw; cd /tmp
  local sh=${SHAPE:-l3_3x3}
  timeout -k 10 120 python -u $R/tools/wgrad_pmc.py > $R/gpurun_out/pmcw/${sh}_time.txt 2>&1 || die pmcw-time
  cat $R/gpurun_out/pmcw/${sh}_time.txt
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
    SQ_INSTS_LDS SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/gpurun_out/pmcw/${sh}_p1 -o run -- \
    python $R/tools/wgrad_pmc.py > $R/gpurun_out/pmcw/p1.log 2>&1 || die pmcw-p1 $R/gpurun_out/pmcw/p1.log
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD \
    GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmcw/${sh}_p2 -o run -- \
    python $R/tools/wgrad_pmc.py > $R/gpurun_out/pmcw/p2.log 2>&1 || die pmcw-p2 $R/gpurun_out/pmcw/p2.log
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv \
    -d $R/gpurun_out/pmcw/${sh}_p3 -o run -- python $R/tools/wgrad_pmc.py > $R/gpurun_out/pmcw/p3.log 2>&1 || die pmcw-p3 $R/gpurun_out/pmcw/p3.log
  cd $R
  python tools/pmc_summary.py gpurun_out/pmcw/${sh}_p1 gpurun_out/pmcw/${sh}_p2 gpurun_out/pmcw/${sh}_p3 2>&1 | tail -40
}
task_pmc_f32() {   # SHAPE / MODE over tools/f32_pmc.py: two PMC passes (waits / LDS / VALU, MFMA busy)
  mkdir -p $R/gpurun_out/pmcf; cd /tmp
  local sh=${SHAPE:-l2_3x3}_${MODE:-fwd}
  timeout -k 10 120 python -u $R/tools/f32_pmc.py > $R/gpurun_out/pmcf/${sh}_time.txt 2>&1 || die pmcf-time
  cat $R/gpurun_out/pmcf/${sh}_time.txt
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
    SQ_INSTS_LDS SQ_INSTS_VALU --kernel-trace --output-format csv -d $R/gpurun_out/pmcf/${sh}_p1 -o run -- \
    python $R/tools/f32_pmc.py > $R/gpurun_out/pmcf/p1.log 2>&1 || die pmcf-p1 $R/gpurun_out/pmcf/p1.log
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD \
    GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmcf/${sh}_p2 -o run -- \
    python $R/tools/f32_pmc.py > $R/gpurun_out/pmcf/p2.log 2>&1 || die pmcf-p2 $R/gpurun_out/pmcf/p2.log
  cd $R
  python tools/pmc_summary.py gpurun_out/pmcf/${sh}_p1 gpurun_out/pmcf/${sh}_p2 2>&1 | tail -40
}
task_f32() {
  timeout -k 10 300 python -u tools/f32_conv_micro.py ${F32B:-64} > ${O}_f32_micro.txt 2>&1 || die f32-micro ${O}_f32_micro.txt
  cat ${O}_f32_micro.txt
  timeout -k 10 300 python -u tools/f32_conv_micro.py 1 > ${O}_f32_micro_b1.txt 2>&1 || die f32-micro-b1 ${O}_f32_micro_b1.txt
  cat ${O}_f32_micro_b1.txt
  PCMP_PHASE_TIMES=1 timeout -k 10 400 python -u pytorch_training_inference.py --models resnet50 --dtype fp32 --synthetic \
    --json ${O}_f32_repro.json > ${O}_f32_repro.txt 2>&1 || die f32-repro ${O}_f32_repro.txt
  grep -E "phase times|Training time|p50|Inference" ${O}_f32_repro.txt | cut -c1-300
}

[ $# -ge 1 ] || { sed -n '2,27p' "$0"; exit 2; }
for t in "$@"; do
  echo "== $t"
  f=task_${t//-/_}
  declare -F $f > /dev/null || { echo "unknown task $t"; exit 2; }
  $f || exit 1
done
