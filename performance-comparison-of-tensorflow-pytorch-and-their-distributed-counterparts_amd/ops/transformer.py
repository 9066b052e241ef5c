"""LayerNorm / GELU / tanh / attention autograd Functions (BERT-base path)."""
from __future__ import annotations

import torch

from .functions import dropout_rng
from .kernels import K
from . import params as _params
from .params import compute_weight, compute_weight_t, emit_grad, sink_or_temp


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


def _partial_rows_grad(p, src2d, n):
    """Gradient of a table parameter whose first ``n`` elements get the column sums of ``src2d``
    (``K.colsum``) and whose other rows get none (BERT's position rows past S, token-type rows > 0).
    Those rows are zeroed on every first write of an accumulation window (one small fill), so no
    state carried across steps -- a shorter S, an in-place edit of the flat gradient, a loaded
    gradient -- can leave a stale value there."""
    def compute(out, acc):
        flat = out.view(-1)
        K.colsum(src2d, flat[:n], acc)
        if flat.numel() > n and not acc:
            flat[n:].zero_()
    return emit_grad(p, compute)


class EmbedLayerNormFn(torch.autograd.Function):
    """BERT embeddings: y = LayerNorm(word_rows + position[:S] (broadcast over the batch) +
    token_type[0]) in one kernel (``embed_layernorm_fwd``, csrc/transformer.hip), reading the
    position / token-type rows from the bf16 shadow.  Backward: the LayerNorm backward kernel, then
    the position gradient as the column sums of dx over the batch and the token-type gradient as
    its column sums over every row (``colsum``) -- no broadcast / cast / add launches of eager torch.
    HF parity: ``BertEmbeddings`` with ``token_type_ids=None`` (pytorch_on_language_distr.py:151-161)."""

    @staticmethod
    def forward(ctx, w_rows, position, token_type, gamma, beta, eps, S):
        dt = w_rows.dtype
        pos = compute_weight(position, dt)[:S].contiguous()
        tt = compute_weight(token_type, dt)[0].contiguous()
        y, xs, mean, rstd = K.embed_layernorm_fwd(w_rows.contiguous(), pos, tt, gamma.detach(), beta.detach(), eps)
        ctx.save_for_backward(xs, mean, rstd)
        ctx.params, ctx.S = (position, token_type, gamma, beta), S
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, mean, rstd = ctx.saved_tensors
        position, token_type, gamma, beta = ctx.params
        gout, acc, fin = sink_or_temp(gamma)
        bout, bacc, bfin = sink_or_temp(beta)
        dx = K.layernorm_bwd(dy.contiguous(), xs, mean, rstd, gamma.detach(), gout, bout, acc or bacc)
        gg, gb = fin(), bfin()
        D, S = dx.shape[-1], ctx.S
        B = dx.numel() // (S * D)
        gp = _partial_rows_grad(position, dx.reshape(B, S * D), S * D)
        gt = _partial_rows_grad(token_type, dx.reshape(B * S, D), D)
        return dx, gp, gt, gg, gb, None, None


def layer_norm(x, gamma, beta, eps, resid=None):
    return LayerNormFn.apply(x, resid, gamma, beta, eps)


def gelu(x):
    return GeluFn.apply(x)


def tanh(x):
    return TanhFn.apply(x)


def attention(qkv, ids, B, S, H, p_drop=0.0):
    return AttentionFn.apply(qkv, ids, B, S, H, p_drop)


# ------------------------------------------------------------------------------------------------
# Fused BERT sublayers.  Each post-LN sublayer of BertLayer is ONE autograd node whose backward
# issues the kernels itself, so that the fusions that cross op boundaries are possible:
#   * dropout(sublayer output) + residual add + LayerNorm: one forward kernel (layernorm_fwd with
#     p), one backward kernel (layernorm_bwd_fused) that also emits the dropped branch's gradient and
#     the bias gradient of the projection that produced it (no dropout / colsum launches);
#   * the residual gradient is added in the epilogue of the sublayer input's DGRAD GEMM (no
#     autograd-engine at::add of the two gradients of h);
#   * GELU: in the epilogue of the FFN up-projection (forward: out = gelu(u), u kept) and of the
#     down-projection's DGRAD (backward: du = (df W2) * gelu'(u)).
# Reference: BertLayer = BertAttention(BertSelfAttention + BertSelfOutput) + BertIntermediate +
# BertOutput of the HF model the reference fine-tunes (pytorch_on_language_distr.py:151-161).

def _dgrad(dy, w, wt, resid=None):
    M, N = dy.shape
    C = w.shape[1]
    return K.conv_dgrad(dy.reshape(M, 1, 1, N), w.reshape(N, 1, 1, C), 1, 1, 1, 0,
                        None if resid is None else resid.reshape(M, 1, 1, C), wt).reshape(M, C)


def _wgrad(p, dy, x):
    M, N = dy.shape
    C = x.shape[1]
    return emit_grad(p, lambda out, acc: K.conv_wgrad(dy.reshape(M, 1, 1, N), x.reshape(M, 1, 1, C), out, 1, 1, 1, 0,
                                                        acc))


def _side_ok(p, t):
    return (t.is_cuda and p.requires_grad and getattr(p, "main_grad", None) is not None and
            _params.side_stream_enabled())


def _wgrad_bias(p, bias, dy, x):
    """Weight gradient dy^T x and bias gradient colsum(dy) of one Linear.  With flat gradient sinks
    they run on the WGRAD side stream (ops/params.py run_on_side), concurrent with the DGRAD /
    attention / LayerNorm-backward chain that only needs dy -- the same split as the conv blocks.
    Returns (grad_w, grad_b) for autograd (None when written into a sink)."""
    if _side_ok(p, dy) and (bias is None or _side_ok(bias, dy)):
        def run():
            _wgrad(p, dy, x)
            if bias is not None:
                emit_grad(bias, lambda o, acc: K.colsum(dy, o, acc))
        _params.run_on_side(run, (dy, x), linear=True)
        return None, None
    gw = _wgrad(p, dy, x)
    gb = emit_grad(bias, lambda o, acc: K.colsum(dy, o, acc)) if bias is not None else None
    return gw, gb


class _SideBatch:
    """The weight / bias gradients of one sublayer backward, issued to the WGRAD side stream as ONE
    ``run_on_side`` fork (the host cost of a fork is on the eager step's critical path:
    profiles/r4_bert_host_prof.txt); without flat sinks / side stream each runs inline at once."""

    def __init__(self):
        self.jobs, self.keep = [], []

    def add(self, p, bias, dy, x):
        if _side_ok(p, dy) and (bias is None or _side_ok(bias, dy)):
            self.jobs.append((p, bias, dy, x))
            self.keep += [dy, x]
            return None, None
        return _wgrad_bias(p, bias, dy, x)

    def flush(self):
        if not self.jobs:
            return
        jobs = self.jobs

        def run():
            for p, bias, dy, x in jobs:
                _wgrad(p, dy, x)
                if bias is not None:
                    emit_grad(bias, lambda o, acc, dy=dy: K.colsum(dy, o, acc))
        _params.run_on_side(run, tuple(self.keep), linear=True)
        self.jobs, self.keep = [], []


def _ln_bwd(ctx, dy, xs, mean, rstd, gamma, beta, bias):
    """-> (dresid, dbranch); gamma / beta / the branch bias gradients emitted."""
    p, seed, off, salt = ctx.ln
    outs, fins, accmask = [], [], 0
    for w, prm in enumerate((gamma, beta, bias)):
        out, acc, fin = sink_or_temp(prm)
        outs.append(out)
        fins.append(fin)
        accmask |= int(bool(acc)) << w
    dx, dxd = K.layernorm_bwd_fused(dy.contiguous(), xs, mean, rstd, gamma.detach(), outs[0], outs[1], outs[2],
                                    accmask, p, seed, off, salt)
    return dx, dxd, [fin() for fin in fins]


class BertAttentionBlockFn(torch.autograd.Function):
    """h1 = LayerNorm(h + dropout(attn_out(attention(qkv(h)))))."""

    @staticmethod
    def forward(ctx, h, ids, wqkv, bqkv, wo, bo, gamma, beta, B, S, H, p_attn, p_hid, eps):
        # one native op for the four kernels (qkv GEMM, attention, out GEMM, dropout+residual+LN):
        # one Python -> C++ dispatch per sublayer on the host-bound eager path
        dt = h.dtype
        wq, wo_c = compute_weight(wqkv, dt), compute_weight(wo, dt)
        seed, off = dropout_rng.next(B * H * S * S) if p_attn > 0 else (0, 0)
        seed_h, off_h = dropout_rng.next(h.numel()) if p_hid > 0 else (0, 0)
        salt = dropout_rng.salt if (p_attn > 0 or p_hid > 0) else None
        y, qkv, out, lse, xs, mean, rstd = K.bert_attn_fwd(
            h.contiguous(), ids, wq, bqkv.detach().float(), wo_c, bo.detach().float(), gamma.detach(), beta.detach(),
            B, S, H, p_attn, seed, off, p_hid, seed_h, off_h, eps, salt)
        ctx.ln = (p_hid, seed_h, off_h, salt if p_hid > 0 else None)
        ctx.save_for_backward(h, qkv, out, lse, ids if ids is not None else torch.empty(0), xs, mean, rstd)
        ctx.attn = (B, S, H, p_attn, seed, off, ids is not None, salt)
        ctx.params = (wqkv, bqkv, wo, bo, gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        h, qkv, out, lse, ids, xs, mean, rstd = ctx.saved_tensors
        wqkv, bqkv, wo, bo, gamma, beta = ctx.params
        B, S, H, p, seed, off, has_ids, salt = ctx.attn
        dt = h.dtype
        if dy.dtype != dt:
            dy = dy.to(dt)
        dres, da, (gg, gb, gbo) = _ln_bwd(ctx, dy, xs, mean, rstd, gamma, beta, bo)
        side = _SideBatch()
        gwo, _ = side.add(wo, None, da, out)
        dctx = _dgrad(da, compute_weight(wo, dt), compute_weight_t(wo, dt))
        dqkv = K.attention_bwd(dctx, qkv, out, lse, ids if has_ids else None, B, S, H, p, seed, off, salt)
        gwq, gbq = side.add(wqkv, bqkv, dqkv, h)
        side.flush()
        dh = _dgrad(dqkv, compute_weight(wqkv, dt), compute_weight_t(wqkv, dt), dres) if ctx.needs_input_grad[0] else None
        return dh, None, gwq, gbq, gwo, gbo, gg, gb, None, None, None, None, None, None


class BertFFNBlockFn(torch.autograd.Function):
    """h2 = LayerNorm(h1 + dropout(ffn2(gelu(ffn1(h1)))))."""

    @staticmethod
    def forward(ctx, h1, w1, b1, w2, b2, gamma, beta, p_hid, eps):
        dt = h1.dtype
        w1c, w2c = compute_weight(w1, dt), compute_weight(w2, dt)
        seed_h, off_h = dropout_rng.next(h1.numel()) if p_hid > 0 else (0, 0)
        salt = dropout_rng.salt if p_hid > 0 else None
        y, g, u, xs, mean, rstd = K.bert_ffn_fwd(h1.contiguous(), w1c, b1.detach().float(), w2c, b2.detach().float(),
                                                 gamma.detach(), beta.detach(), p_hid, seed_h, off_h, eps, salt)
        ctx.ln = (p_hid, seed_h, off_h, salt)
        ctx.save_for_backward(h1, g, u, xs, mean, rstd)
        ctx.params = (w1, b1, w2, b2, gamma, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        h1, g, u, xs, mean, rstd = ctx.saved_tensors
        w1, b1, w2, b2, gamma, beta = ctx.params
        dt = h1.dtype
        if dy.dtype != dt:
            dy = dy.to(dt)
        dres, df, (gg, gb, gb2) = _ln_bwd(ctx, dy, xs, mean, rstd, gamma, beta, b2)
        side = _SideBatch()
        gw2, _ = side.add(w2, None, df, g)
        du = K.linear_dgrad_gelu(df, compute_weight(w2, dt), u, compute_weight_t(w2, dt))
        gw1, gb1 = side.add(w1, b1, du, h1)
        side.flush()
        dh1 = _dgrad(du, compute_weight(w1, dt), compute_weight_t(w1, dt), dres) if ctx.needs_input_grad[0] else None
        return dh1, gw1, gb1, gw2, gb2, gg, gb, None, None
