"""Autograd Functions for the dense / loss / regularisation ops (Linear as a 1x1 implicit-GEMM
conv, Dropout with a counter-based RNG, fused softmax cross-entropy, log-softmax).

Reference parity: the transfer heads ``Linear(2048,512)-ReLU-Dropout(0.2)-Linear(512,10)-
LogSoftmax`` / ``Linear(4096,256)-ReLU-Dropout(0.4)-Linear(256,10)-LogSoftmax`` with
``NLLLoss`` (another_neural_net.py:108-113,250-257), VGG16 classifier FCs with Dropout(0.5)
and the BERT pooler/classifier (pytorch_on_language_distr.py:151-161).
"""
from __future__ import annotations

import itertools

import torch

from .kernels import K
from .params import compute_weight, compute_weight_t, emit_grad


class _RNG:
    """Dropout seed/offset stream: deterministic given ``torch.initial_seed()``.

    ``salt`` (set by :class:`pcmp.engine.graph.GraphedStep` while it captures a training step) is
    a device int64 counter that the dropout / attention kernels mix into the seed; the captured step
    increments it, so every replay of the graph draws new masks although the kernels' arguments
    are frozen at capture time.  Eager steps leave it None."""

    def __init__(self):
        self.seed = None
        self.counter = itertools.count()
        self.salt = None

    def next(self, n: int):
        if self.seed is None:
            self.seed = int(torch.initial_seed()) & ((1 << 62) - 1)
        off = next(self.counter) << 32
        return self.seed, off

    def reseed(self, seed: int):
        self.seed = int(seed) & ((1 << 62) - 1)
        self.counter = itertools.count()


dropout_rng = _RNG()


class LinearFn(torch.autograd.Function):
    """y = act(x @ W^T + b), x [M, Cin] (compute dtype), W [Nout, Cin] fp32 master."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        M, Cin = x.shape
        Nout = weight.shape[0]
        w = compute_weight(weight, x.dtype)
        b = bias.detach().float() if bias is not None else None

        # a plain GEMM on the MFMA kernels: torch.ops.pcmp.conv_fwd plans the kernel / K-split per
        # shape (csrc/igemm.hip plan_gemm); bias and ReLU are fused into the epilogue
        y = K.conv_fwd(x.reshape(M, 1, 1, Cin), w.reshape(Nout, 1, 1, Cin), 1, 0, b, None, relu,
                       False)[0].reshape(M, Nout)
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(x, y)
            ctx.weight, ctx.bias, ctx.relu = weight, bias, relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        weight, bias = ctx.weight, ctx.bias
        dy = dy.contiguous()
        if dy.dtype != x.dtype:
            dy = dy.to(x.dtype)
        if ctx.relu:
            dy = K.relu_bwd(dy, y)
        M, Cin = x.shape
        Nout = weight.shape[0]
        dy4 = dy.reshape(M, 1, 1, Nout)
        x4 = x.reshape(M, 1, 1, Cin)
        gw = emit_grad(weight, lambda out, acc: K.conv_wgrad(dy4, x4, out, 1, 1, 1, 0, acc))
        gb = emit_grad(bias, lambda out, acc: K.colsum(dy, out, acc)) if bias is not None else None
        dx = None
        if ctx.needs_input_grad[0]:
            w = compute_weight(weight, dy.dtype)
            dx = K.conv_dgrad(dy4, w.reshape(Nout, 1, 1, Cin), 1, 1, 1, 0, None,
                              compute_weight_t(weight, dy.dtype)).reshape(M, Cin)
        return dx, gw, gb, None


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        seed, off = dropout_rng.next(x.numel())
        ctx.cfg = (p, seed, off, dropout_rng.salt)
        return K.dropout(x.contiguous(), p, seed, off, dropout_rng.salt)

    @staticmethod
    def backward(ctx, dy):
        p, seed, off, salt = ctx.cfg
        return K.dropout(dy.contiguous(), p, seed, off, salt), None


class SoftmaxXentFn(torch.autograd.Function):
    """mean over valid rows of -log_softmax(z)[y]  (== LogSoftmax + NLLLoss)."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        need = ctx.needs_input_grad[0]
        logits = logits.contiguous()
        r = K.softmax_xent(logits, labels, False, need, 1.0, ignore_index)
        lm = K.loss_mean(r[0], labels.contiguous(), logits.shape[1], ignore_index)   # [mean, valid rows]
        if need:
            ctx.save_for_backward(r[1], lm)
        return lm[0]

    @staticmethod
    def backward(ctx, gout):
        dl, lm = ctx.saved_tensors
        return K.xent_grad_scale(dl, gout.reshape(1).to(torch.float32).contiguous(), lm[1:2]), None, None


class LogSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z):
        r = K.softmax_xent(z.contiguous(), None, True, False, 1.0, -100)
        logp = r[1]
        ctx.save_for_backward(logp)
        ctx.dtype = z.dtype
        return logp

    @staticmethod
    def backward(ctx, g):
        (logp,) = ctx.saved_tensors
        # the g - exp(logp) * sum(g) math runs at g's precision (fp32 from an fp32 NLL); only the
        # result is cast to the activation dtype
        if g.dtype != ctx.dtype and g.dtype != torch.float32:
            g = g.float()
        dz = K.log_softmax_bwd(g.contiguous(), logp)
        return dz if dz.dtype == ctx.dtype else dz.to(ctx.dtype)


def linear(x, weight, bias=None, relu=False):
    return LinearFn.apply(x, weight, bias, relu)


def dropout(x, p, training=True):
    if not training or p == 0.0:
        return x
    return DropoutFn.apply(x, p)


def cross_entropy(logits, labels, ignore_index=-100):
    return SoftmaxXentFn.apply(logits, labels, ignore_index)


def log_softmax(z):
    return LogSoftmaxFn.apply(z)
