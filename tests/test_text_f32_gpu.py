"""fp32 text path on HIP (``--dtype fp32``, the reference's precision: its BERT fine-tune is fp32 end to
end, /root/reference/pytorch_on_language_distr.py:151-161,258-275).  Every text op has an fp32 HIP
kernel (csrc/text_f32.hip); these tests check them op by op against the PyTorch fp32 reference of
the same op (ops/ref.py), and whole-model gradients (BERT 2-layer, BiLSTM) of the HIP fp32 path
against the PyTorch fp32 run of the same model at 1e-4 relative error."""
import pytest
import torch

import pcmp  # noqa: F401
from pcmp.ops import _lib, ref
from pcmp.ops.kernels import FP32_REF_OPS

pytestmark = pytest.mark.gpu


def _ops():
    return torch.ops.pcmp


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def test_no_fp32_reference_fallback():
    assert len(FP32_REF_OPS) == 0


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_layernorm_f32(gpu, p):
    torch.manual_seed(0)
    M, D = 300, 768
    x, r = torch.randn(M, D, device=gpu), torch.randn(M, D, device=gpu)
    g, b = torch.rand(D, device=gpu) + 0.5, torch.randn(D, device=gpu)
    got = _ops().layernorm_fwd(x, r, g, b, 1e-12, p, 7, 11)
    exp = ref.layernorm_fwd(x, r, g, b, 1e-12, p, 7, 11)
    for a, e in zip(got, exp):
        assert a.dtype == torch.float32
        assert _rel(a, e) < 1e-5
    dy = torch.randn(M, D, device=gpu)
    outs = [torch.zeros(D, device=gpu) for _ in range(3)]
    outr = [torch.zeros(D, device=gpu) for _ in range(3)]
    gd = _ops().layernorm_bwd_fused(dy, got[1], got[2], got[3], g, outs[0], outs[1], outs[2], 0, p, 3, 5)
    ed = ref.layernorm_bwd_fused(dy, exp[1], exp[2], exp[3], g, outr[0], outr[1], outr[2], 0, p, 3, 5)
    assert _rel(gd[0], ed[0]) < 1e-5 and _rel(gd[1], ed[1]) < 1e-5
    for a, e in zip(outs, outr):
        assert _rel(a, e) < 1e-5


def test_embed_layernorm_f32(gpu):
    torch.manual_seed(1)
    S, D = 64, 256
    x, pos, tt = torch.randn(4 * S, D, device=gpu), torch.randn(S, D, device=gpu), torch.randn(D, device=gpu)
    g, b = torch.rand(D, device=gpu), torch.randn(D, device=gpu)
    for a, e in zip(_ops().embed_layernorm_fwd(x, pos, tt, g, b, 1e-12), ref.embed_layernorm_fwd(x, pos, tt, g, b, 1e-12)):
        assert _rel(a, e) < 1e-5


@pytest.mark.parametrize("S", [128, 256, 137])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_f32(gpu, p, S):
    """fp32 attention incl. S > 128 (up to 132 KB of dynamic LDS: the kernels opt in to > 64 KB)."""
    torch.manual_seed(2)
    B, H = 3, 4
    D = 64 * H
    qkv = torch.randn(B * S, 3 * D, device=gpu)
    ids = torch.randint(1, 100, (B, S), device=gpu)
    ids[1, 70:] = 0
    ids[2, 5:] = 0
    ctx, lse = _ops().attention_fwd(qkv, ids, B, S, H, p, 9, 3)
    rc, rl = ref.attention_fwd(qkv, ids, B, S, H, p, 9, 3)
    assert _rel(ctx, rc) < 1e-5 and _rel(lse, rl) < 1e-6
    dctx = torch.randn_like(ctx)
    got = _ops().attention_bwd(dctx, qkv, ctx, lse, ids, B, S, H, p, 9, 3)
    exp = ref.attention_bwd(dctx, qkv, rc, rl, ids, B, S, H, p, 9, 3)
    assert _rel(got, exp) < 1e-5


def test_act_embedding_pooling_f32(gpu):
    torch.manual_seed(3)
    x = torch.randn(1000, 64, device=gpu)
    dy = torch.randn_like(x)
    assert _rel(_ops().gelu_fwd(x), ref.gelu_fwd(x)) < 1e-6
    assert _rel(_ops().gelu_bwd(dy, x), ref.gelu_bwd(dy, x)) < 1e-6
    y = _ops().tanh_fwd(x)
    assert _rel(y, ref.tanh_fwd(x)) < 1e-6
    assert _rel(_ops().tanh_bwd(dy, y), ref.tanh_bwd(dy, y)) < 1e-6
    assert _rel(_ops().add_bf16(x, dy), x + dy) == 0.0
    W = torch.randn(500, 32, device=gpu)
    ids = torch.randint(0, 500, (6, 40), device=gpu)
    ids[:, 30:] = 0
    assert torch.equal(_ops().embedding_fwd(ids, W), W[ids])
    g = torch.randn(6, 40, 32, device=gpu)
    dW, dWr = torch.zeros_like(W), torch.zeros_like(W)
    _ops().embedding_bwd(ids, g, dW, 0, False)
    ref.embedding_bwd(ids, g, dWr, 0, False)
    assert _rel(dW, dWr) < 1e-6
    xs = torch.randn(6, 40, 32, device=gpu)
    assert _rel(_ops().masked_mean_fwd(xs, ids), ref.masked_mean_fwd(xs, ids)) < 1e-6
    d2 = torch.randn(6, 32, device=gpu)
    assert _rel(_ops().masked_mean_bwd(d2, ids, 40), ref.masked_mean_bwd(d2, ids, 40)) < 1e-6


def test_lstm_seq_f32(gpu):
    torch.manual_seed(4)
    B, S, H = 9, 40, 64
    gx = torch.randn(B, S, 2, 4 * H, device=gpu)
    whh = torch.randn(2, 4 * H, H, device=gpu) * 0.1
    ids = torch.randint(1, 50, (B, S), device=gpu)
    ids[3, 25:] = 0
    ids[5, :3] = 0
    got = _ops().lstm_seq_fwd(gx, whh, ids)
    exp = ref.lstm_seq_fwd(gx, whh, ids)
    for a, e in zip(got[:3], exp[:3]):
        assert _rel(a, e) < 1e-5
    dh = torch.randn(B, S, 2 * H, device=gpu)
    gd = _ops().lstm_seq_bwd(dh, got[1], got[2], whh, ids)[0]
    ed = ref.lstm_seq_bwd(dh, exp[1], exp[2], whh, ids)[0]
    assert _rel(gd, ed) < 1e-5


def _grads_fp32(model, fn, backend):
    from pcmp.ops.functions import dropout_rng
    dropout_rng.reseed(1234)
    _lib.set_backend(backend)
    old = model.compute_dtype
    model.compute_dtype = torch.float32
    try:
        for p in model.parameters():
            p.grad = None
        loss = fn()
        loss.backward()
        torch.cuda.synchronize()
        return loss.item(), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
    finally:
        model.compute_dtype = old
        _lib.set_backend("hip")


def _check_model(m, fn, label, tol=1e-4):
    lr, gr = _grads_fp32(m, fn, "torch")
    lh, gh = _grads_fp32(m, fn, "hip")
    errs = sorted(((_rel(gh[n], gr[n]), n) for n in gr if gr[n].norm() > 0), reverse=True)
    print(label, "loss torch-fp32 %.7f hip-fp32 %.7f" % (lr, lh), "worst", errs[:3])
    assert set(gh) == set(gr)
    assert abs(lh - lr) <= 1e-5 * max(1.0, abs(lr))
    assert errs[0][0] < tol, errs[:3]


@pytest.mark.parametrize("drop", [0.0, 0.1])
def test_bert2_fp32_grads_match_torch_fp32(gpu, drop):
    from pcmp.models.bert import BertConfig, BertForSequenceClassification
    torch.manual_seed(0)
    m = BertForSequenceClassification(BertConfig(num_hidden_layers=2, hidden_dropout_prob=drop,
                                                 attention_probs_dropout_prob=drop)).to(gpu).train()
    g = torch.Generator(device=gpu).manual_seed(2)
    ids = torch.randint(1000, 30522, (8, 128), device=gpu, generator=g)
    for i, L in enumerate([128, 100, 50, 7, 128, 64, 32, 90]):
        ids[i, L:] = 0
    y = torch.randint(0, 2, (8,), device=gpu, generator=g)
    _check_model(m, lambda: m(ids, None, (ids > 0).long(), y)[0], f"bert2 drop={drop}")


def test_bilstm_fp32_grads_match_torch_fp32(gpu):
    from pcmp.models.bilstm import BiLSTMClassifier
    from pcmp.ops import cross_entropy
    torch.manual_seed(0)
    m = BiLSTMClassifier(2000, 128, 128, 2, 2, 0.0).to(gpu).train()
    g = torch.Generator(device=gpu).manual_seed(1)
    ids = torch.randint(1, 2000, (40, 64), device=gpu, generator=g)
    ids[:, 50:] = 0
    ids[3, 20:] = 0
    y = torch.randint(0, 2, (40,), device=gpu, generator=g)
    _check_model(m, lambda: cross_entropy(m.forward_logits(ids), y), "bilstm")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_embedding_bwd_deterministic(gpu, dtype):
    """Embedding backward (segmented over the stably sorted ids, one writer per vocabulary row) is
    bitwise reproducible across runs and equals the fp64 index_add reference; padding rows skipped;
    knob emb_atomic=1 (the fp32-atomic kernel) matches it to rounding."""
    torch.manual_seed(5)
    V, E, B, S = 300, 64, 8, 40
    ids = torch.randint(0, V, (B, S), device=gpu)
    ids[:, 30:] = 0
    ids[0, :10] = 7                      # a long segment of one id
    dy = torch.randn(B, S, E, device=gpu).to(dtype)
    outs = []
    for _ in range(3):
        dW = torch.full((V, E), 0.5, device=gpu)
        _ops().embedding_bwd(ids, dy, dW, 0, True)
        outs.append(dW)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    # the fixed order: per id, fp32 adds over its rows in row order, then one add into dW (the
    # packed-key sort path must reproduce the stable-sort order exactly)
    dyc, idl = dy.reshape(-1, E).float().cpu(), ids.flatten().tolist()
    exp = torch.full((V, E), 0.5)
    for v in sorted(set(idl) - {0}):
        acc = torch.zeros(E)
        for r, x in enumerate(idl):
            if x == v:
                acc = acc + dyc[r]
        exp[v] = exp[v] + acc
    assert torch.equal(outs[0].cpu(), exp)
    # more rows than the one-workgroup sort takes (16,384): the library stable sort, same bits per run
    big = torch.randint(1, V, (4, 5000), device=gpu)
    dyb = torch.randn(4, 5000, E, device=gpu).to(dtype)
    r1, r2 = torch.zeros(V, E, device=gpu), torch.zeros(V, E, device=gpu)
    _ops().embedding_bwd(big, dyb, r1, 0, True)
    _ops().embedding_bwd(big, dyb, r2, 0, True)
    assert torch.equal(r1, r2)
    keep = (ids.flatten() != 0)
    ref = torch.zeros(V, E, dtype=torch.float64, device=gpu).index_add_(
        0, ids.flatten()[keep], dy.reshape(-1, E)[keep].double()) + 0.5
    torch.testing.assert_close(outs[0].double(), ref, rtol=1e-5, atol=1e-4)
    old = _ops().set_knob("emb_atomic", 1)
    try:
        dW = torch.full((V, E), 0.5, device=gpu)
        _ops().embedding_bwd(ids, dy, dW, 0, True)
    finally:
        _ops().set_knob("emb_atomic", old)
    torch.testing.assert_close(dW, outs[0], rtol=1e-5, atol=1e-5)
