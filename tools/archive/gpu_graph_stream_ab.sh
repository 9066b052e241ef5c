set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed 's/$/ eager forks/' || exit 1
PCMP_WGRAD_STREAM=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>/dev/null | grep -o '"value": [0-9.]*' | sed 's/$/ eager single-stream/' || exit 1
PCMP_WGRAD_STREAM=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --graph 2>/dev/null | grep -o '"value": [0-9.]*' | sed 's/$/ graph single-stream/' || exit 1
done
