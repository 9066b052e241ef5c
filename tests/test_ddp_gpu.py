"""Multi-rank data-parallel rehearsal on ONE GPU (the round-end 8-GPU run is the driver's):
two ranks share cuda:0 and all-reduce CUDA gradient buckets over gloo, exercising the HIP kernels,
the flat-bucket DDP engine and the bench.py rank/aggregation logic end to end."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("kind", ["mlp", "bilstm", "resnet_syncbn"])
def test_ddp_equivalence_on_gpu(gpu, tmp_path, kind):
    from pcmp.parallel.selftest import ddp_equivalence_worker
    os.environ["PYTHONPATH"] = ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")
    mp.spawn(ddp_equivalence_worker, args=(2, _port(), str(tmp_path), kind, 0.01, "cuda"), nprocs=2, join=True)
    for r in range(2):
        res = torch.load(tmp_path / f"rank{r}.pt", weights_only=True)
        assert res["ok_grad"], res
        assert res["ok_sync"], res
        assert res["nbuckets"] >= 2


def test_bench_two_ranks_shared_gpu(gpu):
    env = dict(os.environ, PCMP_DIST_BACKEND="gloo", PCMP_SHARED_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch-size", "16"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 32
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
