"""Cross-rank metric aggregation.

The reference prints per-rank numbers with no aggregation.  Here one all-reduce of a small fp64
vector (sum of losses, correct predictions, sample counts, max wall time) gives global epoch
metrics; rank 0 prints them.  Works over RCCL (GPU tensor) or gloo (CPU tensor).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.kernels import argmax_rows


def _device():
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_sum(values):
    """values: list of floats -> list of global sums."""
    t = torch.tensor(list(values), dtype=torch.float64, device=_device())
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def all_reduce_max(value: float) -> float:
    t = torch.tensor([value], dtype=torch.float64, device=_device())
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class MetricAccumulator:
    """Accumulate on device (no per-step host sync), reduce once per epoch."""

    def __init__(self, device):
        self.device = device
        self.reset()

    def reset(self):
        self.loss_sum = torch.zeros((), dtype=torch.float64, device=self.device)
        self.correct = torch.zeros((), dtype=torch.float64, device=self.device)
        self.count = torch.zeros((), dtype=torch.float64, device=self.device)
        self.steps = 0

    def update(self, loss: torch.Tensor, logits: torch.Tensor | None = None, labels: torch.Tensor | None = None):
        n = labels.numel() if labels is not None else 1
        self.loss_sum += loss.detach().double() * n
        if logits is not None and labels is not None:
            self.correct += (argmax_rows(logits.detach()) == labels).sum().double()
        self.count += n
        self.steps += 1

    def global_values(self):
        s = all_reduce_sum([float(self.loss_sum), float(self.correct), float(self.count)])
        loss = s[0] / max(1.0, s[2])
        acc = s[1] / max(1.0, s[2])
        return {"loss": loss, "accuracy": acc, "samples": int(s[2])}
