"""Flat parameter / gradient / compute-shadow storage ("memory laid out for HBM").

All trainable parameters of a model are re-homed into one fp32 buffer (64-B aligned slices),
their gradients into one fp32 buffer, and their bf16 compute copies into one bf16 buffer:
  * the optimizer step is ONE fused kernel over the whole model (pcmp.optim),
  * DDP buckets are contiguous slices of the gradient buffer — no gather/scatter copies around
    the RCCL all-reduce (pcmp.parallel.ddp),
  * backward kernels write weight gradients straight into ``p.main_grad`` (pcmp.ops.params).
Parameters updated by plain torch autograd (``p.grad``) are folded into ``main_grad`` by a
post-accumulate-grad hook, so torch-native layers interoperate.

Layout order is REVERSE registration order by default: gradients of the last layers arrive
first in backward, so the first DDP bucket fills (and starts its all-reduce) earliest.
"""
from __future__ import annotations

import os

import torch

ALIGN = 16  # elements (64 B fp32) — every slice starts on a 16-byte vector boundary for bf16 too


class FlatParams:
    def __init__(self, params, shadow_dtype=torch.bfloat16, reverse=True, device=None):
        params = [p for p in params if p.requires_grad]
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = list(reversed(uniq)) if reverse else uniq
        if not self.params:
            raise ValueError("FlatParams: no trainable parameters")
        dev = device or self.params[0].device
        self.offsets, off = [], 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.device = dev
        self.master = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.shadow = torch.zeros(off, dtype=shadow_dtype, device=dev) if shadow_dtype is not None else None
        self._hooks = []
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            view = self.master[o:o + n].view_as(p)
            view.copy_(p.detach().to(device=dev, dtype=torch.float32))
            p.data = view
            p.main_grad = self.grad[o:o + n].view_as(p)
            if self.shadow is not None:
                p._shadow = self.shadow[o:o + n].view_as(p)
            p._grad_fresh = True
            self._hooks.append(p.register_post_accumulate_grad_hook(self._fold_torch_grad))
        self._init_transposed()
        self.refresh_shadows()

    # ----------------------------------------------------------------------------------------
    def _init_transposed(self):
        """DGRAD consumes every conv weight as [C][R][S][K].  Instead of one transpose launch per
        DGRAD call, all 4-D weights get a transposed bf16 copy in one more flat buffer, refreshed by
        ONE batched launch (``wt_transpose_multi``) the first time backward asks for it after the
        weights changed (keyed on the global weight generation)."""
        self.shadow_t, self._t_desc, self._t_blocks, self._t_gen = None, None, 0, None
        if self.shadow is None or self.shadow.dtype != torch.bfloat16:
            return
        rows, off, blocks = [], 0, 0
        for p, o in zip(self.params, self.offsets):
            if p.dim() == 4:
                K, R, S, C = p.shape
            elif p.dim() == 2 and getattr(p, "_pcmp_dgrad_t", False):   # Linear weight [Nout, Cin]
                (K, C), R, S = p.shape, 1, 1
            else:
                continue
            tiles = ((K + 63) // 64) * ((C + 63) // 64)
            pad = getattr(p, "_pcmp_s2_pad", None)
            if pad is not None and R > 1 and S > 1 and os.environ.get("PCMP_S2_CLASS_T", "1") != "0":
                # stride-2 conv: the four sub-pixel classes (oph, opw) of its DGRAD one after another,
                # each [C][subR][subS][K] (the layout csrc/igemm.hip dgrad_impl slices; no per-call
                # transpose of the class taps)
                coff = 0
                for oph in (0, 1):
                    for opw in (0, 1):
                        r0, s0 = (oph + pad) & 1, (opw + pad) & 1
                        sub_r, sub_s = (R - r0 + 1) // 2, (S - s0 + 1) // 2
                        rows.append([o, off + coff, K, sub_r * sub_s, C, blocks, S, R * S, r0, s0, 2, sub_s])
                        blocks += sub_r * sub_s * tiles
                        coff += C * sub_r * sub_s * K
                p._t_slice = (off, (p.numel(),))
            else:
                rows.append([o, off, K, R * S, C, blocks, S, R * S, 0, 0, 1, S])
                p._t_slice = (off, (C, R, S, K))
                blocks += R * S * tiles
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        if not rows:
            return
        self.shadow_t = torch.empty(off, dtype=torch.bfloat16, device=self.device)
        self._t_desc = torch.tensor(rows, dtype=torch.int64, device=self.device)
        self._t_blocks = blocks
        for p in self.params:
            sl = getattr(p, "_t_slice", None)
            if sl is not None:
                o, shp = sl
                p._shadow_t = self.shadow_t[o:o + p.numel()].view(shp)
                p._flat_owner = self

    def transposed(self, p):
        """[C,R,S,K] bf16 compute weight of a conv weight ``p`` (batched refresh when stale); for a
        stride-2 conv weight (``_pcmp_s2_pad``) the 1-D class-blocked layout instead."""
        from ..ops.params import WEIGHT_GEN
        if self._t_gen != WEIGHT_GEN[0]:
            from ..ops.kernels import K
            K.wt_transpose_multi(self.shadow, self.shadow_t, self._t_desc, self._t_blocks)
            self._t_gen = WEIGHT_GEN[0]
        return p._shadow_t

    # ----------------------------------------------------------------------------------------
    @staticmethod
    def _fold_torch_grad(p):
        """A torch-native op produced p.grad: move it into the flat buffer and announce it."""
        if p.grad is None:
            return
        if getattr(p, "_grad_fresh", True):
            p.main_grad.copy_(p.grad)
        else:
            p.main_grad.add_(p.grad)
        p.grad = None
        p._grad_fresh = False
        hook = getattr(p, "_grad_ready_hook", None)
        if hook is not None:
            hook(p)

    def refresh_shadows(self):
        from ..ops.params import bump_weight_gen
        bump_weight_gen()
        if self.shadow is not None:
            from ..ops.kernels import K
            K.cast_to_bf16(self.master, self.shadow) if self.shadow.dtype == torch.bfloat16 \
                else self.shadow.copy_(self.master)

    def zero_grad(self):
        """Start a new accumulation window: the next backward write of each param overwrites.
        Slices of params that were never written since the last zero_grad are zeroed so a
        skipped parameter never carries a stale gradient into the optimizer."""
        for p in self.params:
            if getattr(p, "_grad_fresh", True):
                p.main_grad.zero_()
            p._grad_fresh = True

    def slices(self):
        return [(p, o, p.numel()) for p, o in zip(self.params, self.offsets)]

    def state_dict(self):
        return {"numel": self.numel}

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
