"""Process bootstrap: rank/world discovery, process-group init, device binding, device report.

Reference parity: ``--local_rank`` CLI arg injected by the legacy launcher
(another_neural_net.py:63-66, pytorch_on_language_distr.py:20-23), ``init_process_group('gloo')``
(:69 / :26) and the device report strings (another_neural_net.py:83-92).  MI355X-native
differences: one process per GPU, backend ``nccl`` (= RCCL over xGMI on ROCm) whenever GPUs are
used, ``gloo`` for CPU runs; torchrun's ``LOCAL_RANK``/``RANK``/``WORLD_SIZE`` env vars are read
as well as ``--local_rank``; a finite collective timeout plus async error handling so a dead rank
aborts the job instead of hanging.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None

    @property
    def is_main(self):
        return self.rank == 0

    @property
    def distributed(self):
        return self.world_size > 1


def env_ranks(local_rank_arg: int | None = None):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lr_env = os.environ.get("LOCAL_RANK")
    local = int(lr_env) if lr_env is not None else (local_rank_arg if local_rank_arg is not None else 0)
    return rank, world, local


def init(local_rank_arg: int | None = None, backend: str | None = None, timeout_s: float = 600.0,
         use_gpu: bool | None = None, force_init: bool = False) -> DistEnv:
    """Initialise the process group if launched with WORLD_SIZE>1 (or ``force_init``)."""
    rank, world, local = env_ranks(local_rank_arg)
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    # Rehearsal overrides (multi-rank logic on a one-GPU box): PCMP_SHARED_DEVICE=1 binds every
    # rank to cuda:0, PCMP_DIST_BACKEND=gloo selects gloo (RCCL needs one GPU per rank).
    dev_index = 0 if os.environ.get("PCMP_SHARED_DEVICE") == "1" else local
    backend = backend or os.environ.get("PCMP_DIST_BACKEND") or None
    if use_gpu:
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    be = None
    if (world > 1 or force_init) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        # RCCL's internal streams at high priority: its ring kernels hold only a few CUs, and a
        # high-priority queue lets their workgroups start between the conv grids of backward
        os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        be = backend or ("nccl" if use_gpu else "gloo")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    elif dist.is_initialized():
        be = dist.get_backend()
        rank, world = dist.get_rank(), dist.get_world_size()
    return DistEnv(rank, world, local, device, be)


def device_report(local_rank: int = 0, printer=print) -> torch.device:
    """The reference's device banner (another_neural_net.py:83-92), verbatim strings."""
    if torch.cuda.is_available():
        printer("Cuda Device Available")
        printer(list(range(torch.cuda.device_count())))
        device = torch.device("cuda", local_rank)
        printer("Name of the Cuda Device: ", torch.cuda.get_device_name())
        printer("GPU Computational Capablity: ", torch.cuda.get_device_capability())
    else:
        device = torch.device("cpu", local_rank)
        printer("No GPU. switching to CPU")
    return device


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def shutdown():
    if dist.is_initialized():
        dist.destroy_process_group()
