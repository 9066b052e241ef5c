"""ShardedSampler must reproduce torch.utils.data.DistributedSampler bit for bit."""
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler

import pcmp  # noqa: F401
from pcmp.parallel.sampler import ShardedSampler


@pytest.mark.parametrize("n,world,shuffle,drop_last", [(10, 3, True, False), (10, 3, False, False), (9000, 8, True, False),
                                                        (7, 4, True, True), (5, 8, True, False), (1000, 2, False, True)])
def test_matches_distributed_sampler(n, world, shuffle, drop_last):
    for epoch in (0, 3):
        for rank in range(world):
            ref = DistributedSampler(list(range(n)), num_replicas=world, rank=rank, shuffle=shuffle, seed=0,
                                     drop_last=drop_last)
            ref.set_epoch(epoch)
            mine = ShardedSampler(n, num_replicas=world, rank=rank, shuffle=shuffle, seed=0, drop_last=drop_last)
            mine.set_epoch(epoch)
            assert list(ref) == list(mine)
            assert len(ref) == len(mine)


def test_index_list_semantics_and_reference_bug():
    idx = [40, 41, 42, 43, 44, 45]
    good = list(ShardedSampler(idx, num_replicas=2, rank=0, shuffle=False))
    assert good == [40, 42, 44]
    bug = list(ShardedSampler(idx, num_replicas=2, rank=0, shuffle=False, reference_index_bug=True))
    assert bug == [0, 2, 4]   # another_neural_net.py:53-60 behaviour (positions, not indices)


def test_set_epoch_changes_order_unless_frozen():
    a = ShardedSampler(100, 1, 0)
    e0 = list(a)
    a.set_epoch(1)
    assert list(a) != e0
    b = ShardedSampler(100, 1, 0, freeze_epoch=True)
    b.set_epoch(1)
    assert list(b) == e0


def test_shards_partition_dataset():
    n, world = 1001, 8
    seen = []
    for r in range(world):
        seen += list(ShardedSampler(n, world, r, shuffle=True))
    assert set(seen) == set(range(n)) and len(seen) == 1008
