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


def test_ddp_bucket_timeline_shared_gpu(gpu, tmp_path):
    """Two ranks on cuda:0, CUDA buckets over gloo: the first buckets' all-reduces are launched from
    the comm stream while backward still runs (negative launch time relative to the end of
    backward in comm_report's bucket timeline), and average_buffers equalises the BN statistics."""
    from pcmp.parallel.selftest import bucket_timeline_worker
    os.environ["PYTHONPATH"] = ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")
    mp.spawn(bucket_timeline_worker, args=(2, _port(), str(tmp_path), "cuda"), nprocs=2, join=True)
    for r in range(2):
        d = torch.load(tmp_path / f"tl{r}.pt", weights_only=True)
        tl = d["rep"]["bucket_timeline"]
        assert len(tl) == d["rep"]["buckets"] >= 3, d["rep"]
        assert tl[0]["launch_ms"] < 0, tl            # first bucket launched before backward ended
        assert all(t["done_ms"] >= t["launch_ms"] and t["bytes"] > 0 for t in tl), tl
        assert d["differ_before"] and d["equal_after"] and d["is_mean"], d


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
