"""GPU numerics of the BiLSTM / BERT kernels against their PyTorch references, plus model-level
HIP-vs-reference checks for BiLSTM, BERT and VGG16."""
import pytest
import torch

import pcmp  # noqa: F401
from pcmp.ops import _lib, ref

pytestmark = pytest.mark.gpu


def ops():
    return torch.ops.pcmp


def close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"max err {err} > {lim}"


def _ids(B, S, V, dev, lens=None):
    ids = torch.randint(1, V, (B, S), device=dev)
    lens = lens or [S - (7 * i) % S for i in range(B)]
    for i, l in enumerate(lens):
        ids[i, max(1, l):] = 0
    return ids


def test_embedding_and_masked_mean(gpu):
    ids = _ids(6, 40, 500, gpu)
    W = torch.randn(500, 64, device=gpu).to(torch.bfloat16)
    close(ops().embedding_fwd(ids, W), ref.embedding_fwd(ids, W), 0, 0)
    dy = torch.randn(6, 40, 64, device=gpu).to(torch.bfloat16)
    d1 = torch.zeros(500, 64, device=gpu)
    d2 = torch.zeros(500, 64, device=gpu)
    ops().embedding_bwd(ids, dy, d1, 0, False)
    ref.embedding_bwd(ids, dy, d2, 0, False)
    close(d1, d2, 1e-4, 1e-3)
    x = torch.randn(6, 40, 64, device=gpu).to(torch.bfloat16)
    close(ops().masked_mean_fwd(x, ids), ref.masked_mean_fwd(x, ids))
    g = torch.randn(6, 64, device=gpu).to(torch.bfloat16)
    close(ops().masked_mean_bwd(g, ids, 40), ref.masked_mean_bwd(g, ids, 40))


@pytest.mark.parametrize("B,S,H", [(5, 40, 64), (32, 128, 256)])
def test_lstm_recurrence(gpu, B, S, H):
    torch.manual_seed(0)
    ids = _ids(B, S, 1000, gpu)
    gx = (torch.randn(B, S, 2, 4 * H, device=gpu) * 0.5).to(torch.bfloat16)
    whh = (torch.randn(2, 4 * H, H, device=gpu) / H ** 0.5).to(torch.bfloat16)
    h, g, c, sync = ops().lstm_seq_fwd(gx, whh, ids)
    hr, gr, cr, _ = ref.lstm_seq_fwd(gx, whh, ids)
    torch.cuda.synchronize()
    assert int(sync[2].item()) == 0, "barrier timeout"
    close(h, hr, 3e-2, 3e-2)
    close(c, cr, 3e-2, 3e-2)
    dh = torch.randn(B, S, 2 * H, device=gpu).to(torch.bfloat16)
    dg, sync2 = ops().lstm_seq_bwd(dh, g, c, whh, ids)
    dgr, _ = ref.lstm_seq_bwd(dh, gr, cr, whh, ids)
    torch.cuda.synchronize()
    assert int(sync2[2].item()) == 0, "barrier timeout"
    close(dg, dgr, 5e-2, 5e-2)


@pytest.mark.parametrize("B,S,H", [(5, 40, 64), (32, 128, 256), (17, 33, 32)])
def test_lstm_v2_bitwise(gpu, B, S, H):
    """The role-split recurrences (knob lstm_v2: exchange wave + IO waves) run the round-1 kernels'
    arithmetic: every output bitwise equal to lstm_v2 = 0."""
    torch.manual_seed(1)
    ids = _ids(B, S, 1000, gpu)
    gx = (torch.randn(B, S, 2, 4 * H, device=gpu) * 0.5).to(torch.bfloat16)
    whh = (torch.randn(2, 4 * H, H, device=gpu) / H ** 0.5).to(torch.bfloat16)
    dh = torch.randn(B, S, 2 * H, device=gpu).to(torch.bfloat16)
    outs = []
    old = ops().set_knob("lstm_v2", 0)
    try:
        for v in (0, 1):
            ops().set_knob("lstm_v2", v)
            h, g, c, sync = ops().lstm_seq_fwd(gx, whh, ids)
            dg, sync2 = ops().lstm_seq_bwd(dh, g, c, whh, ids)
            torch.cuda.synchronize()
            assert int(sync[2].item()) == 0 and int(sync2[2].item()) == 0, "barrier timeout"
            outs.append((h, g, c, dg))
    finally:
        ops().set_knob("lstm_v2", old)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,S,H", [(5, 40, 64), (32, 128, 256), (17, 33, 32), (8, 16, 512)])
def test_lstm_bwd_partial_exchange(gpu, B, S, H):
    """lstm_v2 = 2: the backward hands off fp32 partial products instead of the dgates tile -- same
    math, another fp32 summation order, so equal to the v2 kernel's dgates to bf16 rounding."""
    torch.manual_seed(2)
    ids = _ids(B, S, 1000, gpu)
    gx = (torch.randn(B, S, 2, 4 * H, device=gpu) * 0.5).to(torch.bfloat16)
    whh = (torch.randn(2, 4 * H, H, device=gpu) / H ** 0.5).to(torch.bfloat16)
    dh = torch.randn(B, S, 2 * H, device=gpu).to(torch.bfloat16)
    old = ops().set_knob("lstm_v2", 1)
    try:
        h, g, c, sync = ops().lstm_seq_fwd(gx, whh, ids)
        dg1, s1 = ops().lstm_seq_bwd(dh, g, c, whh, ids)
        ops().set_knob("lstm_v2", 2)
        dg3, s3 = ops().lstm_seq_bwd(dh, g, c, whh, ids)
        dg3b, _ = ops().lstm_seq_bwd(dh, g, c, whh, ids)
        torch.cuda.synchronize()
    finally:
        ops().set_knob("lstm_v2", old)
    assert int(s1[2].item()) == 0 and int(s3[2].item()) == 0, "barrier timeout"
    assert torch.equal(dg3, dg3b), "partial exchange must be run-to-run deterministic"
    close(dg3, dg1, 5e-2, 5e-2)
    rel = (dg3.float() - dg1.float()).norm() / dg1.float().norm()
    assert rel < 1e-2, rel


def test_layernorm_act(gpu):
    x = torch.randn(300, 768, device=gpu).to(torch.bfloat16)
    r = torch.randn(300, 768, device=gpu).to(torch.bfloat16)
    g = torch.rand(768, device=gpu) + 0.5
    b = torch.randn(768, device=gpu)
    y, xs, m, s = ops().layernorm_fwd(x, r, g, b, 1e-12)
    yr, xsr, mr, sr = ref.layernorm_fwd(x, r, g, b, 1e-12)
    close(y, yr)
    close(xs, xsr, 0, 1e-2)
    dy = torch.randn(300, 768, device=gpu).to(torch.bfloat16)
    dg1, db1, dg2, db2 = (torch.zeros(768, device=gpu) for _ in range(4))
    dx = ops().layernorm_bwd(dy, xs, m, s, g, dg1, db1, False)
    dxr = ref.layernorm_bwd(dy, xsr, mr, sr, g, dg2, db2, False)
    close(dx, dxr)
    close(dg1, dg2, 1e-3, 1e-2)
    close(db1, db2, 1e-3, 1e-2)
    z = torch.randn(64, 3072, device=gpu).to(torch.bfloat16)
    close(ops().gelu_fwd(z), ref.gelu_fwd(z))
    close(ops().gelu_bwd(dy[:64, :768].repeat(1, 4).contiguous(), z), ref.gelu_bwd(dy[:64, :768].repeat(1, 4), z))
    t = ops().tanh_fwd(z)
    close(t, ref.tanh_fwd(z))
    close(ops().tanh_bwd(z, t), ref.tanh_bwd(z, t))


@pytest.mark.parametrize("D", [768, 64])
def test_embed_layernorm_fwd(gpu, D):
    """word rows + position rows broadcast over the batch + one token-type row, then LayerNorm
    (lane-dense kernel at D = 768, generic kernel at D = 64) against the fp32 reference."""
    B, S = 4, 48
    x = torch.randn(B * S, D, device=gpu).to(torch.bfloat16)
    pos = torch.randn(S, D, device=gpu).to(torch.bfloat16)
    tt = torch.randn(D, device=gpu).to(torch.bfloat16)
    g = torch.rand(D, device=gpu) + 0.5
    b = torch.randn(D, device=gpu)
    y, xs, m, s = ops().embed_layernorm_fwd(x, pos, tt, g, b, 1e-12)
    xsf = (x.float().view(B, S, D) + pos.float() + tt.float()).view(B * S, D)
    assert torch.equal(xs, xsf.to(torch.bfloat16))      # (x + pos) + tt in fp32, rounded once
    yr = torch.nn.functional.layer_norm(xs.float(), (D,), g, b, 1e-12)
    close(y, yr)
    yr2, xsr, mr, sr = ref.embed_layernorm_fwd(x, pos, tt, g, b, 1e-12)
    assert torch.equal(xs, xsr)
    close(m, mr, 0, 1e-3)
    close(s, sr, 1e-3, 0)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_layernorm_dropout_fused(gpu, p):
    """LayerNorm(drop(x) + r) forward and the fused backward (dx, dropped-branch grad, dgamma,
    dbeta, bias grad) against the fp32 reference with the same counter-based mask."""
    M, D = 1000, 768
    x = torch.randn(M, D, device=gpu).to(torch.bfloat16)
    r = torch.randn(M, D, device=gpu).to(torch.bfloat16)
    g = torch.rand(D, device=gpu) + 0.5
    b = torch.randn(D, device=gpu)
    salt = torch.tensor([3], device=gpu, dtype=torch.int64)
    y, xs, m, s = ops().layernorm_fwd(x, r, g, b, 1e-12, p, 77, 1 << 32, salt)
    yr, xsr, mr, sr = ref.layernorm_fwd(x, r, g, b, 1e-12, p, 77, 1 << 32, salt)
    close(xs, xsr, 0, 1e-2)
    close(y, yr)
    dy = torch.randn(M, D, device=gpu).to(torch.bfloat16)
    outs = [torch.full((D,), 0.5, device=gpu) for _ in range(6)]
    dx, dxd = ops().layernorm_bwd_fused(dy, xs, m, s, g, outs[0], outs[1], outs[2], 0b100, p, 77, 1 << 32, salt)
    dxr, dxdr = ref.layernorm_bwd_fused(dy, xs, m, s, g, outs[3], outs[4], outs[5], 0b100, p, 77, 1 << 32, salt)
    close(dx, dxr)
    close(dxd, dxdr)
    if p == 0:
        assert dxd.data_ptr() == dx.data_ptr()
    else:
        frac = (dxd == 0).float().mean().item()
        assert abs(frac - p) < 0.02, frac
    for a, c in zip(outs[:3], outs[3:]):
        close(a, c, 1e-3, 1e-2)
    # two outputs only (no bias gradient) and accumulate bits on gamma / beta
    dg, db = torch.ones(D, device=gpu), torch.ones(D, device=gpu)
    ops().layernorm_bwd_fused(dy, xs, m, s, g, dg, db, None, 0b011, p, 77, 1 << 32, salt)
    close(dg, outs[3] + 1, 1e-3, 1e-2)
    close(db, outs[4] + 1, 1e-3, 1e-2)


@pytest.mark.parametrize("M", [4096, 300])
def test_linear_gelu_epilogues(gpu, M):
    """GELU fused into the up-projection's epilogue (out = gelu(u), u kept) and into the
    down-projection's DGRAD epilogue (du = (dy W) * gelu'(u)), planner-chosen kernels / splits."""
    torch.manual_seed(0)
    C, N = 768, 3072
    x = (torch.randn(M, C, device=gpu) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, C, device=gpu) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=gpu) * 0.1
    gl, u = ops().linear_gelu_fwd(x, w, bias)
    glr, ur = ref.linear_gelu_fwd(x, w, bias)
    close(u, ur, 2e-2, 2e-2)
    close(gl, glr, 2e-2, 2e-2)
    w2 = (torch.randn(C, N, device=gpu) * 0.03).to(torch.bfloat16)
    dy = torch.randn(M, C, device=gpu).to(torch.bfloat16)
    du = ops().linear_dgrad_gelu(dy, w2, u)
    dur = ref.linear_dgrad_gelu(dy, w2, u)
    close(du, dur, 2e-2, 2e-2)


@pytest.mark.parametrize("S,p", [(128, 0.0), (128, 0.1), (64, 0.1), (96, 0.0), (32, 0.1)])
def test_attention(gpu, S, p):
    torch.manual_seed(1)
    B, H, D = 3, 12, 768
    qkv = torch.randn(B * S, 3 * D, device=gpu).to(torch.bfloat16)
    ids = _ids(B, S, 30522, gpu, lens=[S, S // 2, 3])
    o, lse = ops().attention_fwd(qkv, ids, B, S, H, p, 99, 5 << 32)
    or_, lser = ref.attention_fwd(qkv, ids, B, S, H, p, 99, 5 << 32)
    close(o, or_)
    close(lse, lser, 1e-3, 1e-3)
    do = torch.randn(B * S, D, device=gpu).to(torch.bfloat16)
    dq = ops().attention_bwd(do, qkv, o, lse, ids, B, S, H, p, 99, 5 << 32)
    dqr = ref.attention_bwd(do, qkv, or_, lser, ids, B, S, H, p, 99, 5 << 32)
    close(dq, dqr, 3e-2, 3e-2)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _grads(model, fn, backend):
    from pcmp.ops.functions import dropout_rng
    dropout_rng.reseed(1234)
    _lib.set_backend(backend)
    try:
        for p in model.parameters():
            p.grad = None
        loss = fn()
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    finally:
        _lib.set_backend("hip")


def test_bilstm_model_native_vs_ref(gpu):
    from pcmp.models.bilstm import BiLSTMClassifier
    from pcmp.ops import cross_entropy
    from pcmp.ops.rnn import check_errors
    torch.manual_seed(0)
    m = BiLSTMClassifier(2000, 128, 128, 2, 2, 0.0).to(gpu).train()
    ids = _ids(40, 64, 2000, gpu)
    y = torch.randint(0, 2, (40,), device=gpu)
    l1, g1 = _grads(m, lambda: cross_entropy(m.forward_logits(ids), y), "hip")
    check_errors()
    l2, g2 = _grads(m, lambda: cross_entropy(m.forward_logits(ids), y), "torch")
    assert abs(l1 - l2) < 2e-2
    for n in g2:
        assert _rel(g1[n], g2[n]) < 0.08, n


def test_bert_model_native_vs_ref(gpu):
    from pcmp.models.bert import BertConfig, BertForSequenceClassification
    torch.manual_seed(0)
    m = BertForSequenceClassification(BertConfig(num_hidden_layers=2, hidden_dropout_prob=0.0,
                                                 attention_probs_dropout_prob=0.0)).to(gpu).train()
    ids = _ids(4, 128, 30522, gpu, lens=[128, 100, 50, 7])
    y = torch.randint(0, 2, (4,), device=gpu)
    l1, g1 = _grads(m, lambda: m(ids, None, (ids > 0).long(), y)[0], "hip")
    l2, g2 = _grads(m, lambda: m(ids, None, (ids > 0).long(), y)[0], "torch")
    assert abs(l1 - l2) < 2e-2
    bad = [(n, _rel(g1[n], g2[n])) for n in g2 if _rel(g1[n], g2[n]) > 0.1]
    assert not bad, bad


def test_vgg16_step(gpu):
    from pcmp.models.vgg import vgg16_transfer
    from pcmp.ops import cross_entropy
    torch.manual_seed(0)
    m = vgg16_transfer().to(gpu).train()
    x = torch.rand(2, 3, 224, 224, device=gpu)
    y = torch.randint(0, 10, (2,), device=gpu)
    l1, g1 = _grads(m, lambda: cross_entropy(m.forward_logits(x), y), "hip")
    l2, g2 = _grads(m, lambda: cross_entropy(m.forward_logits(x), y), "torch")
    assert set(g1) == {n for n, p in m.named_parameters() if p.requires_grad}
    assert abs(l1 - l2) < 5e-2 * max(1, abs(l2))
    # The trainable head is Linear(4096,256)-ReLU-Dropout-Linear(256,10) at batch 2: a hidden unit
    # whose pre-activation sits within bf16 noise of 0 can flip its ReLU between the two bf16
    # paths, which changes that unit's whole fc1 gradient row (seed 0 has a few such units).  Compare
    # per hidden unit and allow at most 4 of 256 flipped units; everything else must agree closely.
    for n in g2:
        a, b = g1[n].float(), g2[n].float()
        if a.dim() == 1:
            a, b = a[:, None], b[:, None]
        row_err = (a - b).norm(dim=1) / (b.norm(dim=1) + 1e-3 * b.norm() + 1e-12)
        assert int((row_err > 0.05).sum()) <= 4, (n, row_err.max().item())


def test_bert_fused_sublayers_native(gpu, monkeypatch):
    """Fused sublayer nodes on the HIP kernels vs the op-by-op layer on the HIP kernels, dropout on
    (same RNG stream): bf16-close loss and gradients."""
    import pcmp.models.bert as bert
    from pcmp.ops.functions import dropout_rng
    ids = _ids(4, 128, 30522, gpu, lens=[128, 100, 50, 7])
    y = torch.randint(0, 2, (4,), device=gpu)
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(bert, "_FUSED", fused)
        torch.manual_seed(0)
        m = bert.BertForSequenceClassification(bert.BertConfig(num_hidden_layers=2)).to(gpu).train()
        dropout_rng.reseed(5)
        loss, _ = m(ids, None, (ids > 0).long(), y)
        loss.backward()
        res[fused] = (loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None})
    assert abs(res[True][0] - res[False][0]) < 2e-2
    bad = [(n, _rel(res[True][1][n], g)) for n, g in res[False][1].items() if _rel(res[True][1][n], g) > 0.05]
    assert not bad, bad


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_bert_fused_sublayer_ops_match_op_sequence(gpu, dtype):
    """bert_attn_fwd / bert_ffn_fwd (one native dispatch per sublayer) == the same kernels issued one op
    at a time (Linear, attention, Linear, dropout + residual + LayerNorm; Linear+GELU, Linear, LN),
    bitwise, with dropout on, in bf16 and fp32."""
    torch.manual_seed(6)
    B, S, H, D, F = 4, 128, 12, 768, 3072
    M = B * S
    o = ops()
    h = (torch.randn(M, D, device=gpu) * 0.5).to(dtype)
    ids = _ids(B, S, 1000, gpu, lens=[128, 90, 33, 5])
    wq, bq = (torch.randn(3 * D, D, device=gpu) * 0.02).to(dtype), torch.randn(3 * D, device=gpu) * 0.02
    wo, bo = (torch.randn(D, D, device=gpu) * 0.02).to(dtype), torch.randn(D, device=gpu) * 0.02
    w1, b1 = (torch.randn(F, D, device=gpu) * 0.02).to(dtype), torch.randn(F, device=gpu) * 0.02
    w2, b2 = (torch.randn(D, F, device=gpu) * 0.02).to(dtype), torch.randn(D, device=gpu) * 0.02
    g, b = torch.rand(D, device=gpu) + 0.5, torch.randn(D, device=gpu) * 0.1

    def lin(x, w, bias):
        return o.conv_fwd(x.view(M, 1, 1, -1), w.view(w.shape[0], 1, 1, -1), 1, 0, bias, None, False, False)[0].view(M, -1)

    fa = o.bert_attn_fwd(h, ids, wq, bq, wo, bo, g, b, B, S, H, 0.1, 11, 3 << 32, 0.1, 11, 4 << 32, 1e-12)
    qkv = lin(h, wq, bq)
    ctx, lse = o.attention_fwd(qkv, ids, B, S, H, 0.1, 11, 3 << 32)
    y = o.layernorm_fwd(lin(ctx, wo, bo), h, g, b, 1e-12, 0.1, 11, 4 << 32)
    for u, v in zip(fa, [y[0], qkv, ctx, lse] + list(y[1:])):
        assert torch.equal(u, v)
    h1 = fa[0]
    ff = o.bert_ffn_fwd(h1, w1, b1, w2, b2, g, b, 0.1, 11, 5 << 32, 1e-12)
    gu, uu = o.linear_gelu_fwd(h1, w1, b1)
    y2 = o.layernorm_fwd(lin(gu, w2, b2), h1, g, b, 1e-12, 0.1, 11, 5 << 32)
    for u, v in zip(ff, [y2[0], gu, uu] + list(y2[1:])):
        assert torch.equal(u, v)
    r = ref.bert_ffn_fwd(h1, w1, b1, w2, b2, g, b, 0.1, 11, 5 << 32, 1e-12)
    close(ff[0], r[0], rtol=5e-2 if dtype == torch.bfloat16 else 1e-3, atol=5e-2 if dtype == torch.bfloat16 else 1e-3)


def test_graphed_bert_step_matches_eager_without_dropout(gpu):
    """GraphedStep (whole training step as one hipGraph) == eager steps bitwise-close when dropout is
    off: same losses over 4 steps with AdamW + clipping + a linear LR schedule run between replays;
    with dropout on, replays draw a new mask every step (device salt) and training still decreases."""
    from pcmp.engine.graph import GraphedStep
    from pcmp.engine.trainer import make_state
    from pcmp.models.bert import BertConfig, BertForSequenceClassification
    from pcmp.optim import linear_schedule_with_warmup
    torch.manual_seed(0)
    cfg = BertConfig(num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    ids = torch.randint(1, 30522, (8, 128), device=gpu)
    ids[:, 100:] = 0
    mask = (ids > 0).long()
    y = torch.randint(0, 2, (8,), device=gpu)
    losses = {}
    for mode in ("eager", "graph"):
        torch.manual_seed(1)
        m = BertForSequenceClassification(cfg).to(gpu)
        st = make_state(m, "adamw", lr=1e-4, eps=1e-8, clip=1.0)
        st.sched = linear_schedule_with_warmup(st.opt, 0, 8)
        fn = lambda a, b, c, m=m: m(a, None, b, c)[0]   # noqa: E731
        out = []
        if mode == "graph":
            g = GraphedStep(st, fn, [ids, mask, y])
            for _ in range(4):
                out.append(float(g(ids, mask, y)))
        else:
            for _ in range(4):
                st.zero_grad()
                loss = fn(ids, mask, y)
                st.backward_step(loss)
                out.append(loss.detach().item())
        losses[mode] = out
    for a, b in zip(losses["eager"], losses["graph"]):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(a)), losses
    # dropout on: masks differ per replay (device salt), loss goes down on a fixed batch
    torch.manual_seed(2)
    m = BertForSequenceClassification(BertConfig(num_hidden_layers=2)).to(gpu)
    st = make_state(m, "adamw", lr=3e-4, eps=1e-8, clip=1.0)
    g = GraphedStep(st, lambda a, b, c: m(a, None, b, c)[0], [ids, mask, y])
    seq = [float(g(ids, mask, y)) for _ in range(12)]
    assert int(g.salt.item()) == 12
    assert min(seq[-3:]) < seq[0], seq
