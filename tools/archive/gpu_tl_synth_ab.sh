set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -x -q -s --timeout 240 --timeout-method thread -k transfer > gpurun_out/tl_native.log 2>&1; grep "TL flow" gpurun_out/tl_native.log
PCMP_SYNTH_NATIVE=0 timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -x -q -s --timeout 240 --timeout-method thread -k transfer > gpurun_out/tl_torch.log 2>&1; grep "TL flow" gpurun_out/tl_torch.log
