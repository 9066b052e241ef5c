"""Model parity on CPU (framework model on the reference-op path vs stock torch.nn / HF)."""
import pytest
import torch

import pcmp
from pcmp.ops import cross_entropy


def _rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-20)).item()


def test_resnet18_matches_torch_nn():
    from pcmp.models.resnet import resnet18
    from pcmp.models.torch_ref import TorchResNet
    torch.manual_seed(0)
    m = resnet18(num_classes=10).train()
    t = TorchResNet("resnet18", 10).train().load_from_pcmp(m)
    x, y = torch.randn(4, 3, 64, 64), torch.randint(0, 10, (4,))
    l = cross_entropy(m.forward_logits(x), y)
    l.backward()
    lt = torch.nn.functional.cross_entropy(t(x), y)
    lt.backward()
    assert abs(l.item() - lt.item()) < 1e-4
    assert _rel(m.stem.conv.weight.grad[..., :3].permute(0, 3, 1, 2), t.conv1.weight.grad) < 1e-3
    assert _rel(m.layer3[0].downsample.weight.grad.permute(0, 3, 1, 2), t.layer3[0].downsample[0].weight.grad) < 1e-3
    assert torch.allclose(m.stem.conv.running_mean, t.bn1.running_mean, atol=1e-5)


@pytest.mark.parametrize("cin,planes,stride", [(64, 64, 1), (256, 128, 2)])
def test_bottleneck_matches_torch(cin, planes, stride):
    from pcmp.models.resnet import Bottleneck
    from pcmp.models.torch_ref import TBottleneck
    torch.manual_seed(0)
    b, t = Bottleneck(cin, planes, stride).train(), TBottleneck(cin, planes, stride).train()
    with torch.no_grad():
        for nm, L in zip("123", b.main_layers()):
            getattr(t, "conv" + nm).weight.copy_(L.weight.permute(0, 3, 1, 2))
        t.downsample[0].weight.copy_(b.downsample.weight.permute(0, 3, 1, 2))
    x = torch.randn(2, cin, 8, 8)
    xp = x.permute(0, 2, 3, 1).contiguous().requires_grad_(True)
    xt = x.clone().requires_grad_(True)
    y, yt = b(xp), t(xt)
    g = torch.randn_like(yt)
    y.backward(g.permute(0, 2, 3, 1))
    yt.backward(g)
    assert torch.allclose(y.permute(0, 3, 1, 2), yt, atol=1e-4)
    assert _rel(xp.grad.permute(0, 3, 1, 2), xt.grad) < 1e-4
    assert _rel(b.conv2.weight.grad.permute(0, 3, 1, 2), t.conv2.weight.grad) < 1e-4


def test_resnet50_param_count_matches_torchvision():
    from pcmp.models.resnet import count_params, resnet50, resnet50_transfer
    assert count_params(resnet50()) == 25557032          # torchvision figure
    m = resnet50_transfer()
    head = sum(p.numel() for p in m.fc.parameters())
    assert count_params(m.fc) == 1054218
    assert all(not p.requires_grad for n, p in m.named_parameters() if not n.startswith("fc."))
    assert head >= 1054218


def test_vgg16_param_count():
    from pcmp.models.resnet import count_params
    from pcmp.models.vgg import vgg16, vgg16_transfer
    assert count_params(vgg16()) == 138357544            # torchvision VGG16
    assert count_params(vgg16_transfer()) == 135311946    # SURVEY §2.4.2 (TL head 1,051,402)


def test_bilstm_matches_torch_lstm():
    from pcmp.models.bilstm import BiLSTMClassifier, TorchBiLSTM
    torch.manual_seed(0)
    t = TorchBiLSTM(500, 32, 16, 2, 2, 0.0)
    m = BiLSTMClassifier(500, 32, 16, 2, 2, 0.0).load_torch_lstm(t.embedding, t.lstm, t.fc)
    ids = torch.randint(1, 500, (4, 12))
    for i, l in enumerate([12, 7, 3, 1]):
        ids[i, l:] = 0
    y = torch.randint(0, 2, (4,))
    l = cross_entropy(m.forward_logits(ids), y)
    l.backward()
    lt = torch.nn.functional.cross_entropy(t(ids), y)
    lt.backward()
    assert abs(l.item() - lt.item()) < 1e-5
    assert _rel(m.layers[0].w_hh.grad[1], t.lstm.weight_hh_l0_reverse.grad) < 1e-4
    assert _rel(m.embedding.weight.grad, t.embedding.weight.grad) < 1e-4


def test_bert_matches_hf():
    transformers = pytest.importorskip("transformers")
    from pcmp.models.bert import BertConfig, BertForSequenceClassification
    torch.manual_seed(0)
    kw = dict(num_hidden_layers=2, hidden_size=64, num_attention_heads=1, intermediate_size=128)
    hf = transformers.BertForSequenceClassification(transformers.BertConfig(num_labels=2, hidden_dropout_prob=0.0,
                                                                            attention_probs_dropout_prob=0.0, **kw))
    m = BertForSequenceClassification(BertConfig(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, **kw)).load_hf(hf)
    ids = torch.randint(1, 30522, (2, 32))
    ids[1, 10:] = 0
    y = torch.tensor([0, 1])
    out = hf(ids, attention_mask=(ids > 0).long(), labels=y)
    loss, logits = m(ids, None, (ids > 0).long(), y)
    assert torch.allclose(logits, out.logits, atol=1e-5)
    out.loss.backward()
    loss.backward()
    sd = dict(hf.named_parameters())
    assert _rel(m.layers[1].ffn1.weight.grad, sd["bert.encoder.layer.1.intermediate.dense.weight"].grad) < 1e-4
    # embeddings (EmbedLayerNormFn): position rows [:S] and token-type row 0 get the summed gradient,
    # the rows no token used stay zero
    hp = sd["bert.embeddings.position_embeddings.weight"].grad
    ht = sd["bert.embeddings.token_type_embeddings.weight"].grad
    assert _rel(m.position.grad[:32], hp[:32]) < 1e-4 and float(m.position.grad[32:].abs().max()) == 0.0
    assert _rel(m.token_type.grad, ht) < 1e-4
    assert _rel(m.emb_ln.weight.grad, sd["bert.embeddings.LayerNorm.weight"].grad) < 1e-4


def test_bert_position_grad_rows_past_s_stay_zero():
    """Flat gradient sinks across windows with S1 < S2 > S3: the position rows no token of the
    current window used hold zero (no stale rows from a longer earlier window)."""
    from pcmp.models.bert import BertConfig, BertForSequenceClassification
    from pcmp.utils.flat import FlatParams
    torch.manual_seed(0)
    m = BertForSequenceClassification(BertConfig(num_hidden_layers=1, hidden_size=64, num_attention_heads=1,
                                                 intermediate_size=128, hidden_dropout_prob=0.0,
                                                 attention_probs_dropout_prob=0.0))
    flat = FlatParams(m.parameters())
    for S in (16, 48, 16):
        flat.zero_grad()
        ids = torch.randint(1, 30522, (2, S))
        m(ids, None, None, torch.tensor([0, 1]))[0].backward()
        g = m.position.main_grad
        assert float(g[:S].abs().max()) > 0
        assert float(g[S:].abs().max()) == 0.0, S
        assert float(m.token_type.main_grad[1:].abs().max()) == 0.0


def test_bert_fused_sublayers_match_op_by_op(monkeypatch):
    """The fused sublayer nodes (dropout+residual+LayerNorm fwd/bwd kernels, GELU and residual-grad
    GEMM epilogues) give the op-by-op layer's loss and gradients, dropout ON (same RNG stream)."""
    import pcmp.models.bert as bert
    from pcmp.ops.functions import dropout_rng
    kw = dict(num_hidden_layers=2, hidden_size=256, num_attention_heads=4, intermediate_size=512)
    ids = torch.randint(1, 30522, (2, 32))
    ids[1, 20:] = 0
    y = torch.tensor([0, 1])
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(bert, "_FUSED", fused)
        torch.manual_seed(0)
        m = bert.BertForSequenceClassification(bert.BertConfig(**kw)).train()
        dropout_rng.reseed(123)
        loss, _ = m(ids, None, (ids > 0).long(), y)
        loss.backward()
        res[fused] = (loss.item(), {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
    assert abs(res[True][0] - res[False][0]) < 1e-5
    assert set(res[True][1]) == set(res[False][1])
    for n, g in res[False][1].items():
        assert _rel(res[True][1][n], g) < 1e-4, n


def test_bert_base_param_count():
    from pcmp.models.bert import bert_base
    from pcmp.models.resnet import count_params
    assert count_params(bert_base()) == 109483778


def test_keras_resnet_and_mlp_head_shapes():
    from pcmp.models.keras_resnet import KerasResNet50TL
    from pcmp.models.layers import MLPHead
    m = KerasResNet50TL(10, image_size=64)
    p = m(torch.rand(2, 3, 64, 64))
    assert p.shape == (2, 10) and torch.allclose(p.sum(1), torch.ones(2), atol=1e-5)
    h = MLPHead(2048, 512, 10, 0.2).eval()
    out = h(torch.randn(3, 2048))
    assert torch.allclose(out.exp().sum(1), torch.ones(3), atol=1e-5)


def test_resnet_eval_mode_uses_running_stats():
    from pcmp.models.resnet import resnet18
    from pcmp.models.torch_ref import TorchResNet
    torch.manual_seed(0)
    m = resnet18(10).train()
    for _ in range(2):
        m.forward_logits(torch.randn(4, 3, 32, 32))
    t = TorchResNet("resnet18", 10).load_from_pcmp(m).eval()
    m.eval()
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        assert torch.allclose(m.forward_logits(x), t(x), atol=1e-4)


def test_bn_folding_cache_invalidates():
    """Eval forwards use BN folded into the conv weights; the cache must follow every weight /
    running-stat change (training forward, fused optimizer step, load_state_dict)."""
    from pcmp.engine.trainer import make_state
    from pcmp.models.resnet import resnet18
    from pcmp.models.torch_ref import TorchResNet
    from pcmp.ops import cross_entropy
    torch.manual_seed(0)
    m = resnet18(10)
    x = torch.randn(2, 3, 32, 32)

    def check():
        m.eval()
        t = TorchResNet("resnet18", 10).load_from_pcmp(m).eval()
        with torch.no_grad():
            assert torch.allclose(m.forward_logits(x), t(x), atol=1e-4)
        m.train()

    check()
    st = make_state(m, "sgd", lr=0.1, momentum=0.9)
    for _ in range(2):
        st.zero_grad()
        st.backward_step(cross_entropy(m.forward_logits(torch.randn(4, 3, 32, 32)), torch.tensor([0, 1, 2, 3])))
        check()
    sd = {k: v.clone() * 1.01 if v.is_floating_point() else v for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    check()


def test_block_boundary_bn_fusion_matches_unfused(monkeypatch):
    """The next block's dgrad epilogue computing this block's BN-backward reduction (and handing
    back the ReLU-masked gradient) must give the same gradients as the separate reduction pass."""
    from pcmp.models.resnet import resnet18, resnet50
    from pcmp.ops import conv_blocks, cross_entropy
    for ctor in (resnet18, resnet50):
        torch.manual_seed(0)
        m = ctor(10)
        x = torch.randn(2, 3, 64, 64)
        y = torch.tensor([1, 2])

        def grads():
            for p in m.parameters():
                p.grad = None
            cross_entropy(m.forward_logits(x), y).backward()
            return [p.grad.clone() for p in m.parameters()]
        g_fused = grads()
        monkeypatch.setattr(conv_blocks, "_link_prev_tail", lambda x: None)
        g_plain = grads()
        monkeypatch.undo()
        for a, b in zip(g_fused, g_plain):
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-6)


def _randomise_bn_stats(tm):
    g = torch.Generator().manual_seed(3)
    for m in tm.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.copy_(torch.randn(m.num_features, generator=g) * 0.1)
            m.running_var.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.weight.data.copy_(torch.rand(m.num_features, generator=g) + 0.5)
            m.bias.data.copy_(torch.randn(m.num_features, generator=g) * 0.1)


@pytest.mark.parametrize("arch", ["resnet18", "resnet50"])
def test_resnet_load_torchvision_state_dict(tmp_path, arch):
    """A torchvision-layout state_dict (TorchResNet has torchvision's module names) saved to disk and
    read back with weights_only=True loads into the framework ResNet: eval logits agree (fp32, CPU)."""
    from pcmp.models import resnet
    from pcmp.models.torch_ref import TorchResNet
    torch.manual_seed(0)
    tm = TorchResNet(arch, 1000).eval()
    _randomise_bn_stats(tm)
    path = tmp_path / "w.pth"
    torch.save(tm.state_dict(), path)
    sd = torch.load(path, weights_only=True)
    m = getattr(resnet, arch)(1000).eval()
    used = m.load_torchvision(sd)
    assert set(used) == {k for k in sd if not k.endswith("num_batches_tracked")}
    x = torch.rand(2, 3, 64, 64)
    with torch.no_grad():
        ref = tm(x)
        out = m(x)
    assert (out - ref).abs().max().item() <= 1e-3 * ref.abs().max().item() + 1e-4


def test_resnet_load_torchvision_into_tl_model():
    """The reference's TL flow: pretrained 1000-way backbone, new MLP head (another_neural_net.py:95-112).
    The 1000-way fc in the file is skipped (its shape does not match the head)."""
    from pcmp.models import resnet
    from pcmp.models.torch_ref import TorchResNet
    tm = TorchResNet("resnet50", 1000)
    m = resnet.resnet50_transfer(10)
    used = m.load_torchvision(tm.state_dict())
    assert "fc.weight" not in used and "layer4.2.bn3.running_var" in used
    assert torch.equal(m.layer4[2].conv3.weight.permute(0, 3, 1, 2), tm.layer4[2].conv3.weight)
