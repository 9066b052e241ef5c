"""Optimizers over :class:`pcmp.utils.flat.FlatParams` (one fused kernel per step) and LR schedules.

Reference parity:
  * ``SGD``   — Keras ``SGD(lr=0.001)`` (resnet.py:24) and the north-star ResNet SGD;
  * ``Adam``  — ``optim.Adam(model.fc.parameters(), lr=0.003)`` (another_neural_net.py:114) and
    ``optim.Adam(model.parameters())`` (:258);
  * ``AdamW`` — HF ``AdamW(lr=2e-5, eps=1e-8)`` (pytorch_on_language_distr.py:167-170; HF's default
    weight_decay 0.0);
  * ``linear_schedule_with_warmup`` — ``get_linear_schedule_with_warmup`` (:182-183);
  * ``clip_grad_norm`` — ``clip_grad_norm_(model.parameters(), 1.0)`` (:271-273), computed on
    device and applied inside the optimizer kernel (no host sync).
LR and step live in device scalars so a captured hipGraph replays correctly across steps.
"""
from __future__ import annotations

import math

import torch

from .ops.kernels import K
from .ops.params import bump_weight_gen
from .utils.flat import FlatParams


class _FlatOptimizer:
    def __init__(self, flat: FlatParams, lr: float):
        self.flat = flat
        dev = flat.device
        self.lr_t = torch.tensor([float(lr)], dtype=torch.float32, device=dev)
        self._lr = float(lr)
        self.base_lr = float(lr)
        self.grad_scale = None   # optional device scalar (clip coef * 1/world)
        self.steps = 0

    @property
    def lr(self):
        return self._lr

    def set_lr(self, lr: float):
        self._lr = float(lr)
        self.lr_t.fill_(self._lr)

    def zero_grad(self, set_to_none: bool = True):
        self.flat.zero_grad()

    def clip_grad_norm(self, max_norm: float, pre_scale: float = 1.0, post_scale: float = 1.0):
        """Global L2 norm of (pre_scale * grad); sets the device-side multiplier
        ``min(1, max_norm/norm) * post_scale`` consumed by the next ``step``.  Returns the norm
        as a device tensor (no sync)."""
        norm, coef = K.grad_clip_coef(self.flat.grad, pre_scale, max_norm, post_scale)
        self.grad_scale = coef
        return norm

    def set_grad_scale(self, scale: float | None):
        if scale is None or scale == 1.0:
            self.grad_scale = None
        else:
            self.grad_scale = torch.tensor([float(scale)], device=self.flat.device)

    # ---- ranged steps: DistributedDataParallel.finish_gradient_sync(opt=...) updates each gradient
    # bucket as soon as its all-reduce completes: begin_step(), step_range() per flat slice, end_step().
    # The same elementwise kernel over a sub-range: bitwise equal to step() over the whole arena.
    def begin_step(self):
        pass

    def step_range(self, lo: int, hi: int):
        raise NotImplementedError

    def end_step(self):
        self.steps += 1
        bump_weight_gen()

    def step(self):
        self.begin_step()
        self.step_range(0, self.flat.numel)
        self.end_step()

    def state_dict(self):
        return {"lr": self._lr, "steps": self.steps, "state": {k: v.detach().clone() for k, v in self._state().items()}}

    def load_state_dict(self, sd):
        self.set_lr(sd["lr"])
        self.steps = sd["steps"]
        for k, v in self._state().items():
            v.copy_(sd["state"][k].to(v.device))

    def _state(self):
        return {}


class SGD(_FlatOptimizer):
    def __init__(self, flat, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(flat, lr)
        self.momentum, self.dampening, self.wd, self.nesterov = momentum, dampening, weight_decay, nesterov
        self.mom = torch.zeros_like(flat.master) if momentum != 0 else flat.master.new_empty(0)

    def step_range(self, lo, hi):
        f = self.flat
        K.sgd_flat(f.master[lo:hi], f.grad[lo:hi], self.mom[lo:hi] if self.mom.numel() else self.mom,
                   f.shadow[lo:hi] if f.shadow is not None else None, None, self.lr_t, self.grad_scale,
                   self.momentum, self.dampening, self.wd, self.nesterov, self.steps == 0)

    def _state(self):
        return {"mom": self.mom}


class Adam(_FlatOptimizer):
    decoupled = False

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(flat, lr)
        self.beta1, self.beta2 = betas
        self.eps, self.wd = eps, weight_decay
        self.m1 = torch.zeros_like(flat.master)
        self.m2 = torch.zeros_like(flat.master)
        self.step_t = torch.zeros(1, dtype=torch.float32, device=flat.device)

    def begin_step(self):
        self.step_t.add_(1.0)

    def step_range(self, lo, hi):
        f = self.flat
        K.adam_flat(f.master[lo:hi], f.grad[lo:hi], self.m1[lo:hi], self.m2[lo:hi],
                    f.shadow[lo:hi] if f.shadow is not None else None, None, self.lr_t, self.grad_scale,
                    self.step_t, self.beta1, self.beta2, self.eps, self.wd, self.decoupled)

    def _state(self):
        return {"m1": self.m1, "m2": self.m2, "step_t": self.step_t}


class AdamW(Adam):
    decoupled = True

    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(flat, lr, betas, eps, weight_decay)


class LambdaLR:
    def __init__(self, opt: _FlatOptimizer, fn):
        self.opt, self.fn, self.last_step = opt, fn, 0
        opt.set_lr(opt.base_lr * fn(0))

    def step(self):
        self.last_step += 1
        self.opt.set_lr(self.opt.base_lr * self.fn(self.last_step))

    def get_last_lr(self):
        return [self.opt.lr]


def linear_schedule_with_warmup(opt, num_warmup_steps, num_training_steps):
    """transformers.get_linear_schedule_with_warmup semantics."""
    def fn(step):
        if step < num_warmup_steps:
            return float(step) / float(max(1, num_warmup_steps))
        return max(0.0, float(num_training_steps - step) / float(max(1, num_training_steps - num_warmup_steps)))
    return LambdaLR(opt, fn)


def cosine_schedule(opt, total_steps, warmup=0):
    def fn(step):
        if step < warmup:
            return step / max(1, warmup)
        return 0.5 * (1 + math.cos(math.pi * min(1.0, (step - warmup) / max(1, total_steps - warmup))))
    return LambdaLR(opt, fn)


def build(name: str, flat: FlatParams, **kw):
    name = name.lower()
    if name == "sgd":
        return SGD(flat, **kw)
    if name == "adam":
        return Adam(flat, **kw)
    if name == "adamw":
        return AdamW(flat, **kw)
    raise ValueError(name)
