set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ew_micro.py > gpurun_out/ew_micro.log 2>&1 || { echo ew_micro failed; tail -30 gpurun_out/ew_micro.log; exit 1; }
cat gpurun_out/ew_micro.log | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kt.log 2>&1 || { echo tests failed; tail -30 gpurun_out/kt.log; exit 1; }
tail -2 gpurun_out/kt.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
