"""Distributed tests without a cluster: gloo, world_size 2, CPU."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import pcmp
from pcmp.parallel.ddp import plan_buckets

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("kind", ["mlp", "bilstm", "resnet_syncbn"])
def test_ddp_equals_single_process(tmp_path, kind):
    from pcmp.parallel.selftest import ddp_equivalence_worker
    os.environ["PYTHONPATH"] = ROOT + os.pathsep + os.environ.get("PYTHONPATH", "")
    world = 2
    mp.spawn(ddp_equivalence_worker, args=(world, _port(), str(tmp_path), kind), nprocs=world, join=True)
    for r in range(world):
        res = torch.load(tmp_path / f"rank{r}.pt", weights_only=True)
        assert res["ok_grad"], res
        assert res["ok_sync"], res
        assert res["nbuckets"] >= 2


def test_plan_buckets_small_first_bucket():
    sizes = [10] * 100
    b = plan_buckets(sizes, 25, 200)
    assert b[0] == (0, 3)                      # first bucket closes at >= 25 elements
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    assert b[-1][1] == 100
    assert sum(e - s for s, e in b) == 100


def test_plan_buckets_small_last_bucket():
    sizes = [10] * 100
    b = plan_buckets(sizes, 25, 200, 35)
    assert b[0] == (0, 3)
    assert b[-1] == (96, 100)                  # tail bucket closes at >= 35 elements from the end
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    assert sum(e - s for s, e in b) == 100
    assert plan_buckets([5], 25, 200, 35) == [(0, 1)]
    assert plan_buckets([10, 10], 25, 200, 100) == [(0, 1), (1, 2)]   # the tail never takes slice 0
