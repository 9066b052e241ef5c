"""Embedding / BiLSTM / masked-mean autograd Functions (BiLSTM text path).

The per-layer BiLSTM node does: one MFMA GEMM for the input projections of both directions and
all timesteps (``W_ih`` stacked [8H, Ein], biases b_ih + b_hh folded into the epilogue), one
persistent recurrence launch (``lstm_seq_fwd``) per 32-sequence chunk; backward: one persistent
BPTT launch per chunk (``lstm_seq_bwd``) producing gate gradients, then weight gradients as MFMA
wgrad GEMMs over all timesteps and the input gradient as one dgrad GEMM.
"""
from __future__ import annotations

import torch

from .kernels import K
from .params import compute_weight, emit_grad

CHUNK = 32  # sequences per persistent-recurrence launch (LB in csrc/rnn.hip)
_pending_sync = []


def check_errors():
    """Synchronise and raise if any persistent recurrence launch hit its spin timeout."""
    global _pending_sync
    for s in _pending_sync:
        if int(s[2].item()) != 0:
            _pending_sync = []
            raise RuntimeError("pcmp LSTM persistent kernel: grid barrier timeout")
    _pending_sync = []


def _track(sync):
    if sync.is_cuda:
        _pending_sync.append(sync)
        if len(_pending_sync) > 256:
            del _pending_sync[:128]


class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, padding_idx, dtype):
        w = compute_weight(weight, dtype)
        ctx.save_for_backward(ids)
        ctx.weight, ctx.padding_idx = weight, padding_idx
        return K.embedding_fwd(ids, w)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        dy = dy.contiguous()
        g = emit_grad(ctx.weight, lambda out, acc: K.embedding_bwd(ids, dy, out, ctx.padding_idx, acc))
        return None, g, None, None


class MaskedMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ids):
        ctx.save_for_backward(ids)
        ctx.S = x.shape[1]
        return K.masked_mean_fwd(x.contiguous(), ids)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        return K.masked_mean_bwd(dy.contiguous(), ids, ctx.S), None


def _hprev(hout, H):
    """Recurrent inputs h_{t-1} (forward order of each direction) as [B,S,2,H]."""
    B, S, _ = hout.shape
    hp = torch.zeros(B, S, 2, H, dtype=hout.dtype, device=hout.device)
    hp[:, 1:, 0] = hout[:, :-1, :H]
    hp[:, :-1, 1] = hout[:, 1:, H:]
    return hp


class BiLSTMLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ids, w_ih, b_ih, b_hh, w_hh):
        B, S, Ein = x.shape
        G8 = w_ih.shape[0]
        H = G8 // 8
        dt = x.dtype
        wih = compute_weight(w_ih, dt)
        whh = compute_weight(w_hh, dt).contiguous()
        bias = (b_ih.detach().float() + b_hh.detach().float())
        x2 = x.reshape(B * S, 1, 1, Ein).contiguous()
        gx = K.conv_fwd(x2, wih.reshape(G8, 1, 1, Ein), 1, 0, bias, None, False, False)[0]
        gx = gx.reshape(B, S, 2, 4 * H)
        outs, gates, cst = [], [], []
        for b0 in range(0, B, CHUNK):
            sl = slice(b0, min(B, b0 + CHUNK))
            h, g, c, sync = K.lstm_seq_fwd(gx[sl].contiguous(), whh, ids[sl].contiguous())
            _track(sync)
            outs.append(h)
            gates.append(g)
            cst.append(c)
        hout = torch.cat(outs) if len(outs) > 1 else outs[0]
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(x, ids, hout)
            ctx.state = (gates, cst)
            ctx.params = (w_ih, b_ih, b_hh, w_hh)
        return hout

    @staticmethod
    def backward(ctx, dh):
        x, ids, hout = ctx.saved_tensors
        gates, cst = ctx.state
        w_ih, b_ih, b_hh, w_hh = ctx.params
        B, S, Ein = x.shape
        G8 = w_ih.shape[0]
        H = G8 // 8
        dt = x.dtype
        whh = compute_weight(w_hh, dt).contiguous()
        dh = dh.contiguous().to(dt)
        dgl = []
        for k, b0 in enumerate(range(0, B, CHUNK)):
            sl = slice(b0, min(B, b0 + CHUNK))
            dg, sync = K.lstm_seq_bwd(dh[sl].contiguous(), gates[k], cst[k], whh, ids[sl].contiguous())
            _track(sync)
            dgl.append(dg)
        dgates = torch.cat(dgl) if len(dgl) > 1 else dgl[0]          # [B,S,2,4H]
        dg2 = dgates.reshape(B * S, 1, 1, G8)
        x2 = x.reshape(B * S, 1, 1, Ein).contiguous()
        g_wih = emit_grad(w_ih, lambda out, acc: K.conv_wgrad(dg2, x2, out, 1, 1, 1, 0, acc))
        g_bih = emit_grad(b_ih, lambda out, acc: K.colsum(dgates.reshape(B * S, G8), out, acc))
        g_bhh = emit_grad(b_hh, lambda out, acc: K.colsum(dgates.reshape(B * S, G8), out, acc))
        hp = _hprev(hout, H)

        def whh_grad(out, acc):
            for d in range(2):
                dgd = dgates[:, :, d].reshape(B * S, 1, 1, 4 * H).contiguous()
                hpd = hp[:, :, d].reshape(B * S, 1, 1, H).contiguous()
                K.conv_wgrad(dgd, hpd, out[d], 1, 1, 1, 0, acc)
        g_whh = emit_grad(w_hh, whh_grad)
        dx = None
        if ctx.needs_input_grad[0]:
            wih = compute_weight(w_ih, dt)
            dx = K.conv_dgrad(dg2, wih.reshape(G8, 1, 1, Ein), 1, 1, 1, 0, None).reshape(B, S, Ein)
        ctx.state = None
        return dx, None, g_wih, g_bih, g_bhh, g_whh
