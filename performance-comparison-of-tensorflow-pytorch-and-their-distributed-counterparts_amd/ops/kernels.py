"""Device dispatch for the native op set.

``K.<op>(*args)`` runs ``torch.ops.pcmp.<op>`` when the first tensor argument lives on the GPU
(raising if the HIP library is missing — see :mod:`pcmp.ops._lib`) and the PyTorch reference
:mod:`pcmp.ops.ref` otherwise.  Both return the same structure.
"""
from __future__ import annotations

import os

import torch

from . import _lib, ref

# PCMP_TRACE_OPS=1 records (op, [shapes]) of every dispatched op in TRACE (profiling aid)
TRACE = [] if os.environ.get("PCMP_TRACE_OPS") else None

OP_NAMES = (
    "conv_fwd", "conv_dgrad", "conv_dgrad_bnr", "conv_wgrad", "conv1x1_bwd_fused",
    "bn_partials", "bn_finalize", "bn_eval_coeff", "bn_apply", "bn_bwd_reduce", "bn_bwd_finalize",
    "bn_bwd_apply",
    "maxpool_fwd", "maxpool_bwd", "maxpool_bwd_bnr", "gap_fwd", "gap_bwd", "softmax_xent", "loss_mean", "xent_grad_scale", "log_softmax_bwd", "dropout", "relu_bwd", "colsum",
    "nchw_to_nhwc", "nchw_to_nhwc_f32", "image_to_s2d", "image_to_s2d_f32", "resize_image",
    "sgd_flat", "adam_flat", "grad_clip_coef", "grad_sumsq_parts", "clip_coef_parts", "cast_to_bf16", "wt_transpose_multi",
    "embedding_fwd", "embedding_bwd", "lstm_seq_fwd", "lstm_seq_bwd",
    "masked_mean_fwd", "masked_mean_bwd",
    "layernorm_fwd", "embed_layernorm_fwd", "layernorm_bwd", "layernorm_bwd_fused", "gelu_fwd", "gelu_bwd",
    "linear_gelu_fwd", "linear_dgrad_gelu", "attention_fwd", "attention_bwd", "tanh_fwd", "tanh_bwd", "add_bf16",
    "topk_rows", "synth_images", "bert_attn_fwd", "bert_ffn_fwd",
)


# Ops that run the PyTorch reference in the fp32 precision mode (``--dtype fp32``).  Empty: every op
# has an fp32 HIP kernel -- the image ops in csrc/f32.hip, the text encoders' (LayerNorm, attention,
# GELU / tanh, embedding, masked mean, BiLSTM recurrence, Linear+GELU) in csrc/text_f32.hip.
FP32_REF_OPS = frozenset()


def _first_tensor(args):
    for a in args:
        if isinstance(a, torch.Tensor):
            return a
    raise TypeError("no tensor argument")


class _Dispatch:
    def __getattr__(self, name):
        refimpl = getattr(ref, name, None)
        fp32_ref = name in FP32_REF_OPS
        native = []   # the resolved torch.ops.pcmp.<name>.default overload (per-call host cost counts)

        def call(*args):
            t = _first_tensor(args)
            if TRACE is not None:
                TRACE.append((name, [tuple(a.shape) if isinstance(a, torch.Tensor) else a for a in args]))
            if _lib.use_native(t) and not (fp32_ref and _lib.precision() == "fp32"):
                if not native:
                    native.append(getattr(torch.ops.pcmp, name).default)
                return native[0](*args)
            if refimpl is None:
                raise NotImplementedError(f"no reference implementation for {name}")
            return refimpl(*args)

        call.__name__ = name
        setattr(self, name, call)
        return call


K = _Dispatch()


def argmax_rows(z: torch.Tensor) -> torch.Tensor:
    """``z.argmax(1)`` of [B, C] scores (native wave-per-row kernel on the GPU)."""
    if z.dim() == 2 and z.stride(1) == 1 and z.dtype in (torch.float32, torch.bfloat16):
        return K.topk_rows(z, 1, False)[0].view(-1)
    return z.argmax(1)


def topk_rows(z: torch.Tensor, k: int):
    """(values fp32, indices) of the k largest scores per row (k <= 8 native; torch otherwise)."""
    if z.dim() == 2 and z.stride(1) == 1 and k <= 8 and z.dtype in (torch.float32, torch.bfloat16):
        return tuple(K.topk_rows(z, k, True))
    v, i = z.float().topk(k, dim=-1)
    return v, i
