"""Data-parallel input sharding.

``ShardedSampler`` reproduces ``torch.utils.data.DistributedSampler`` exactly (same permutation
from ``torch.Generator().manual_seed(seed + epoch)``, padding by repetition to a multiple of the
world size, ``rank::world`` striding, ``drop_last``) — bit-compatible index streams — and adds
what the reference's use lacks: ``set_epoch`` is expected to be called every epoch (the
reference never calls it, so every epoch sees the same order; ``freeze_epoch=True`` restores that
behaviour).  ``reference_index_bug=True`` reproduces another_neural_net.py:53-60, where the
sampler is built over a *list of indices* and therefore yields positions 0..len-1 instead of the
shuffled indices — kept only for parity experiments.
"""
from __future__ import annotations

import math

import torch


class ShardedSampler:
    def __init__(self, data_len_or_indices, num_replicas=None, rank=None, shuffle=True, seed=0, drop_last=False,
                 reference_index_bug=False, freeze_epoch=False):
        import torch.distributed as dist
        if num_replicas is None:
            num_replicas = dist.get_world_size() if dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_initialized() else 0
        if isinstance(data_len_or_indices, int):
            self.indices = None
            n = data_len_or_indices
        else:
            self.indices = list(data_len_or_indices)
            n = len(self.indices)
        self.n, self.world, self.rank = n, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.reference_index_bug = reference_index_bug
        self.freeze_epoch = freeze_epoch
        self.epoch = 0
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int):
        if not self.freeze_epoch:
            self.epoch = epoch

    def positions(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        return idx[self.rank: self.total_size: self.world]

    def __iter__(self):
        pos = self.positions()
        if self.indices is None or self.reference_index_bug:
            return iter(pos)
        return iter(self.indices[i] for i in pos)

    def __len__(self):
        return self.num_samples
