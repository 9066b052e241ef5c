#!/bin/bash
# Round-2 evidence run: model-parity GPU tests (-s, values printed), the notebook flow at the
# reference config (P1/P3/P4: 9,469 images, B=64, 1 epoch of 119 steps + eval + save + reload +
# 1000 batch-1 images, ResNet-50 and VGG16) with per-phase device times, the distributed script's
# VGG16 path (3 epochs, early stopping) under torchrun, and a rocprofv3 kernel summary of VGG16.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${STAGE:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
timeout -k 10 600 python -u -m pytest tests/test_model_parity_gpu.py -v -s --timeout 240 --timeout-method thread > gpurun_out/parity.log 2>&1 || { echo "parity tests failed"; tail -60 gpurun_out/parity.log; exit 1; }
grep -E "rel err|median|convergence|TL flow|loss fp32|passed|failed" gpurun_out/parity.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = repro ]; then
PCMP_PHASE_TIMES=1 timeout -k 10 600 python -u pytorch_training_inference.py --models resnet50,vgg16 --json gpurun_out/repro_nb.jsonl > gpurun_out/repro_nb.log 2>&1 || { echo "notebook flow failed"; tail -40 gpurun_out/repro_nb.log; exit 1; }
grep -E "Epoch|Training time|Inference time|phase" gpurun_out/repro_nb.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=$((29500 + RANDOM % 1000)) another_neural_net.py --model vgg16 --json gpurun_out/repro_vgg_dist.jsonl > gpurun_out/repro_vgg_dist.log 2>&1 || { echo "vgg dist failed"; tail -40 gpurun_out/repro_vgg_dist.log; exit 1; }
grep -E "Epoch|Early|Training time|Inference time" gpurun_out/repro_vgg_dist.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vgg -o run -- python another_neural_net.py --model vgg16 --epochs 1 --train-size 1280 --num-images 100 > gpurun_out/prof_vgg.log 2>&1 || { echo "rocprof vgg failed"; tail -30 gpurun_out/prof_vgg.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_vgg --top 40 > gpurun_out/prof_vgg_summary.txt
head -45 gpurun_out/prof_vgg_summary.txt
find gpurun_out/prof_vgg -name "*kernel_trace.csv" -delete; true
fi
