# round 6: the reference's image flows end to end (pytorch_training_inference.py --models resnet50,vgg16,
# bf16 and the reference's fp32), the BiLSTM / BERT text flow (pytorch_on_language_distr.py), and a
# final rocprof kernel table + stream report of the flagship step
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/r6_reference_repro.txt; : > $O
for dt in bf16 fp32; do
  echo "== --dtype $dt" >> $O
  timeout -k 10 400 python -u pytorch_training_inference.py --models resnet50,vgg16 --synthetic --dtype $dt >> $O 2>&1 || { echo "repro $dt failed"; tail -20 $O; exit 1; }
  grep -E "Training time|Inference time|Test accuracy" $O | tail -6
done
echo "== text: bilstm" >> $O
timeout -k 10 400 python -u pytorch_on_language_distr.py --model bilstm --synthetic >> $O 2>&1 || { echo "text bilstm failed"; tail -20 $O; exit 1; }
grep -E "Training epoch took|Validation Accuracy|Test" $O | tail -4
bash tools/gpu.sh prof-bench
