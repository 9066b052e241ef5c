"""Checkpoint / resume.

Reference: whole-module pickles ``torch.save(model, path)`` / ``torch.load(path)`` hand the trained
TL model to the inference cell and implement VGG's best-by-val-loss early stopping
(pytorch_training_inference_on_image.ipynb:700,852,2093,2104,2120); no optimizer state, no
resume, no rank-0 guard.  Here:
  * ``save_checkpoint`` — model + optimizer + epoch + RNG states as a state_dict, rank 0 only,
    atomic rename; ``load_checkpoint`` restores all of it (resume) with ``weights_only=True``;
  * ``save_model`` / ``load_model`` — the "whole model" hand-off: the constructor spec + state_dict
    (no pickled code objects), so ``load_model(path)`` rebuilds the module standalone;
  * ``BestCheckpoint`` — keep-best-by-metric helper for early stopping.
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch

from .report import is_main


def _atomic_save(obj, path):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def rng_state():
    st = {"torch": torch.get_rng_state(),
          "numpy": torch.from_numpy(np.random.get_state()[1].astype(np.int64)),
          "python": repr(random.getstate())}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    from ..ops.functions import dropout_rng
    st["dropout_seed"] = dropout_rng.seed if dropout_rng.seed is not None else -1
    return st


def save_checkpoint(path, model, optimizer=None, epoch=0, extra=None, all_ranks=False):
    if not (all_ranks or is_main()):
        return
    sd = {"model": model.state_dict(), "epoch": int(epoch), "rng": rng_state()}
    if optimizer is not None and hasattr(optimizer, "state_dict"):
        sd["optimizer"] = optimizer.state_dict()
    if extra:
        sd["extra"] = extra
    _atomic_save(sd, path)


def load_checkpoint(path, model, optimizer=None, map_location="cpu"):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(sd["model"])
    if optimizer is not None and "optimizer" in sd:
        optimizer.load_state_dict(sd["optimizer"])
    rng = sd.get("rng", {})
    if "torch" in rng:
        torch.set_rng_state(rng["torch"])
    if "cuda" in rng and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(rng["cuda"])
    _refresh_flat(model)
    return sd.get("epoch", 0), sd.get("extra")


def _refresh_flat(model):
    """Keep bf16 compute shadows consistent with freshly loaded fp32 masters."""
    seen = set()
    for p in model.parameters():
        sh = getattr(p, "_shadow", None)
        if sh is not None and id(sh) not in seen:
            sh.copy_(p.detach().to(sh.dtype))
            seen.add(id(sh))


def save_model(path, model, spec: dict):
    """Whole-model hand-off: ``spec`` = {"builder": "pcmp.models.resnet:resnet50_transfer", "kwargs": {...}}."""
    if is_main():
        _atomic_save({"spec": spec, "model": model.state_dict()}, path)


def load_model(path, map_location="cpu"):
    import importlib
    sd = torch.load(path, map_location=map_location, weights_only=True)
    mod, fn = sd["spec"]["builder"].split(":")
    if mod.startswith("pcmp."):
        import pcmp  # noqa: F401
    builder = getattr(importlib.import_module(mod), fn)
    model = builder(**sd["spec"].get("kwargs", {}))
    model.load_state_dict(sd["model"])
    return model


class BestCheckpoint:
    def __init__(self, mode="min"):
        self.best = float("inf") if mode == "min" else -float("inf")
        self.mode = mode
        self.state = None

    def update(self, value, model) -> bool:
        better = value < self.best if self.mode == "min" else value > self.best
        if better:
            self.best = value
            self.state = {k: v.detach().clone() for k, v in model.state_dict().items()}
        return better

    def restore(self, model):
        if self.state is not None:
            model.load_state_dict(self.state)
            _refresh_flat(model)
