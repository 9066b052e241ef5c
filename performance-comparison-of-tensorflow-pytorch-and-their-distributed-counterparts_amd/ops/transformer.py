"""LayerNorm / GELU / tanh / attention autograd Functions (BERT-base path)."""
from __future__ import annotations

import torch

from .functions import dropout_rng
from .kernels import K
from .params import sink_or_temp


class LayerNormFn(torch.autograd.Function):
    """y = LayerNorm(x [+ residual]) with fp32 gamma/beta; the residual add is fused."""

    @staticmethod
    def forward(ctx, x, resid, gamma, beta, eps):
        y, xs, mean, rstd = K.layernorm_fwd(x.contiguous(), None if resid is None else resid.contiguous(),
                                            gamma.detach(), beta.detach(), eps)
        ctx.save_for_backward(xs, mean, rstd)
        ctx.gamma, ctx.beta, ctx.has_r = gamma, beta, resid is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, mean, rstd = ctx.saved_tensors
        gout, acc, fin = sink_or_temp(ctx.gamma)
        bout, bacc, bfin = sink_or_temp(ctx.beta)
        dx = K.layernorm_bwd(dy.contiguous(), xs, mean, rstd, ctx.gamma.detach(), gout, bout, acc or bacc)
        gg, gb = fin(), bfin()
        return dx, (dx if ctx.has_r else None), gg, gb, None


class GeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return K.gelu_fwd(x.contiguous())

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return K.gelu_bwd(dy.contiguous(), x)


class TanhFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = K.tanh_fwd(x.contiguous())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return K.tanh_bwd(dy.contiguous(), y)


class AttentionFn(torch.autograd.Function):
    """ctx = softmax(Q K^T / sqrt(64) + mask) [dropout] V over heads of a fused QKV [B*S, 3D]."""

    @staticmethod
    def forward(ctx, qkv, ids, B, S, H, p_drop):
        seed, off = dropout_rng.next(B * H * S * S) if p_drop > 0 else (0, 0)
        salt = dropout_rng.salt if p_drop > 0 else None
        out, lse = K.attention_fwd(qkv.contiguous(), ids, B, S, H, p_drop, seed, off, salt)
        ctx.save_for_backward(qkv, out, lse, ids if ids is not None else torch.empty(0))
        ctx.cfg = (B, S, H, p_drop, seed, off, ids is not None, salt)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse, ids = ctx.saved_tensors
        B, S, H, p, seed, off, has_ids, salt = ctx.cfg
        dqkv = K.attention_bwd(dout.contiguous(), qkv, out, lse, ids if has_ids else None, B, S, H, p, seed, off,
                               salt)
        return dqkv, None, None, None, None, None


def layer_norm(x, gamma, beta, eps, resid=None):
    return LayerNormFn.apply(x, resid, gamma, beta, eps)


def gelu(x):
    return GeluFn.apply(x)


def tanh(x):
    return TanhFn.apply(x)


def attention(qkv, ids, B, S, H, p_drop=0.0):
    return AttentionFn.apply(qkv, ids, B, S, H, p_drop)
