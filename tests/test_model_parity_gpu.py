"""Model-level correctness in regimes where bf16 is close to fp32.

* eval-mode ResNet-50 logits at B=32 against an fp32 torch.nn ResNet-50 with the same weights and
  running statistics (``zero_init_residual=True``: without it a random-init ResNet-50's logits are
  differences of huge activations, and even autocast is 12 % off fp32);
* train-mode ResNet-50 gradients with ``zero_init_residual=True`` at B=64: the per-layer median
  relative error of the HIP path against fp32 must be at most 2x that of stock torch autocast-bf16
  and below an absolute cap;
* BiLSTM / BERT gradients against an fp32 run of the same model: per parameter no worse than the
  bf16 PyTorch-reference path (same bf16 roundings, torch ops) by more than 1.5x;
* convergence parity: ResNet-18 on the learnable synthetic Imagenette-shaped set, 150 steps with
  linear lr warm-up, HIP vs torch autocast: both loss curves fall and end within noise;
* the transfer-learning flow (frozen backbone + MLP head, Adam 3e-3, the notebook's recipe, nb
  :436-446) reaches >= 0.9 test accuracy (the reference's P2 is 0.979, nb :830).
"""
import pytest
import torch

import pcmp
from pcmp.ops import _lib, cross_entropy

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-20)).item()


def _tname(n):
    n = n.replace("stem.conv.weight", "conv1.weight").replace("stem.conv.gamma", "bn1.weight") \
         .replace("stem.conv.beta", "bn1.bias")
    for i in "123":
        n = n.replace(f"conv{i}.gamma", f"bn{i}.weight").replace(f"conv{i}.beta", f"bn{i}.bias")
    return n.replace("downsample.weight", "downsample.0.weight").replace("downsample.gamma", "downsample.1.weight") \
            .replace("downsample.beta", "downsample.1.bias")


def _to_torch_layout(n, g, num_classes):
    if g.dim() == 4:
        g = g[..., :3].permute(0, 3, 1, 2) if n.startswith("stem") else g.permute(0, 3, 1, 2)
    if n.startswith("fc."):
        g = g[:num_classes]
    return g


def _populate_running_stats(m, gpu, res, n=25):
    g = torch.Generator(device=gpu).manual_seed(3)
    m.train()
    with torch.no_grad():
        for _ in range(n):
            m.forward_logits(torch.rand(32, 3, res, res, device=gpu, generator=g))


def test_resnet50_eval_logits_match_fp32(gpu):
    from pcmp.models.resnet import resnet50
    from pcmp.models.torch_ref import TorchResNet
    torch.manual_seed(0)
    m = resnet50(num_classes=1000, zero_init_residual=True).to(gpu)
    _populate_running_stats(m, gpu, 128)
    m.eval()
    x = torch.rand(32, 3, 128, 128, device=gpu, generator=torch.Generator(device=gpu).manual_seed(9))
    with torch.no_grad():
        zh = m.forward_logits(x).float()
        t = TorchResNet("resnet50", 1000).to(gpu).load_from_pcmp(m).eval()
        z32 = t(x).float()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            za = t(x).float()
    e_h, e_a = _rel(zh, z32), _rel(za, z32)
    print(f"eval logits rel err: hip {e_h:.4f} autocast {e_a:.4f}")
    assert e_h < 2 * e_a + 5e-3 and e_h < 0.1, (e_h, e_a)
    assert (zh.argmax(1) == z32.argmax(1)).float().mean() >= 0.9


def test_resnet50_train_grads_per_layer(gpu):
    from pcmp.models.resnet import resnet50
    from pcmp.models.torch_ref import TorchResNet
    torch.manual_seed(0)
    nc = 10
    m = resnet50(num_classes=nc, zero_init_residual=True).to(gpu).train()
    g = torch.Generator(device=gpu).manual_seed(4)
    x = torch.rand(64, 3, 128, 128, device=gpu, generator=g)
    y = torch.randint(0, nc, (64,), device=gpu, generator=g)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    for p in m.parameters():
        p.grad = None
    lh = cross_entropy(m.forward_logits(x), y)
    lh.backward()
    gh = {_tname(n): _to_torch_layout(n, p.grad.float(), nc) for n, p in m.named_parameters()}
    m.load_state_dict(state)
    t = TorchResNet("resnet50", nc).to(gpu).train().load_from_pcmp(m)
    ts = {k: v.clone() for k, v in t.state_dict().items()}
    res = {}
    for mode in ("fp32", "autocast"):
        t.load_state_dict(ts)
        t.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode == "autocast"):
            loss = torch.nn.functional.cross_entropy(t(x).float(), y)
        loss.backward()
        res[mode] = (loss.item(), {n: p.grad.float().clone() for n, p in t.named_parameters()})
    ref = res["fp32"][1]
    names = [n for n in ref if n in gh and ref[n].norm() > 0]
    eh = sorted(_rel(gh[n], ref[n]) for n in names)
    ea = sorted(_rel(res["autocast"][1][n], ref[n]) for n in names)
    med_h, med_a = eh[len(eh) // 2], ea[len(ea) // 2]
    print(f"{len(names)} params; median rel err hip {med_h:.4f} autocast {med_a:.4f}; max hip {eh[-1]:.4f} "
          f"autocast {ea[-1]:.4f}; loss hip {lh.item():.5f} fp32 {res['fp32'][0]:.5f}")
    assert abs(lh.item() - res["fp32"][0]) < 0.01 * abs(res["fp32"][0])
    assert med_h <= 2 * med_a + 2e-3, (med_h, med_a)
    # measured: median 0.172 (HIP) vs 0.173 (autocast) -- train-mode BatchNorm amplifies the bf16
    # rounding of 53 layers for any bf16 implementation; the cap catches a real kernel bug (>> 0.3)
    assert med_h < 0.25, med_h


def _text_grads(model, fn, backend, fp32=False):
    from pcmp.ops.functions import dropout_rng
    dropout_rng.reseed(1234)
    _lib.set_backend(backend)
    old = model.compute_dtype
    model.compute_dtype = torch.float32 if fp32 else None
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


def _bf16_noise_check(m, fn, label):
    l32, g32 = _text_grads(m, fn, "torch", fp32=True)
    lh, gh = _text_grads(m, fn, "hip")
    lr, gr = _text_grads(m, fn, "torch")
    worst = []
    for n in g32:
        if g32[n].norm() == 0:
            continue
        eh, er = _rel(gh[n], g32[n]), _rel(gr[n], g32[n])
        worst.append((eh - 1.5 * er, n, eh, er))
    worst.sort(reverse=True)
    print(label, "loss fp32 %.5f hip %.5f refbf16 %.5f" % (l32, lh, lr), "worst", worst[:3])
    assert abs(lh - l32) < 1e-2
    bad = [(n, eh, er) for d, n, eh, er in worst if eh > 1.5 * er + 5e-3]
    assert not bad, bad


def test_bilstm_grads_at_bf16_noise_level(gpu):
    from pcmp.models.bilstm import BiLSTMClassifier
    from pcmp.ops.rnn import check_errors
    torch.manual_seed(0)
    m = BiLSTMClassifier(2000, 128, 128, 2, 2, 0.0).to(gpu).train()
    g = torch.Generator(device=gpu).manual_seed(1)
    ids = torch.randint(1, 2000, (40, 64), device=gpu, generator=g)
    ids[:, 50:] = 0
    y = torch.randint(0, 2, (40,), device=gpu, generator=g)
    _bf16_noise_check(m, lambda: cross_entropy(m.forward_logits(ids), y), "bilstm")
    check_errors()


def test_bert_grads_at_bf16_noise_level(gpu):
    from pcmp.models.bert import BertConfig, BertForSequenceClassification
    torch.manual_seed(0)
    m = BertForSequenceClassification(BertConfig(num_hidden_layers=2, hidden_dropout_prob=0.0,
                                                 attention_probs_dropout_prob=0.0)).to(gpu).train()
    g = torch.Generator(device=gpu).manual_seed(2)
    ids = torch.randint(1000, 30522, (8, 128), device=gpu, generator=g)
    for i, L in enumerate([128, 100, 50, 7, 128, 64, 32, 90]):
        ids[i, L:] = 0
    y = torch.randint(0, 2, (8,), device=gpu, generator=g)
    _bf16_noise_check(m, lambda: m(ids, None, (ids > 0).long(), y)[0], "bert")


def test_resnet18_convergence_parity_with_autocast(gpu):
    """pcmp (bitwise deterministic) and torch autocast train the same ResNet-18 from the same weights
    on the same batches.  At lr 0.05 the autocast reference itself was bimodal across runs (last-20
    mean loss 0.000-0.99 over six runs on one box, MIOpen algorithm choice varies run to run), so
    the comparison runs at lr 0.02 with MIOpen's deterministic algorithms."""
    from pcmp.data.synthetic import SyntheticImages
    from pcmp.models.resnet import resnet18
    from pcmp.models.torch_ref import TorchResNet
    from pcmp.optim import SGD
    from pcmp.utils.flat import FlatParams
    steps, B, res, lr0, warm = 150, 64, 64, 0.02, 30
    det = (torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    ds = SyntheticImages(steps * B, 10, res, seed=5, device=gpu)
    batches = [ds.get_batch(list(range(i * B, (i + 1) * B))) for i in range(steps)]
    torch.manual_seed(0)
    m = resnet18(num_classes=10).to(gpu).train()
    t = TorchResNet("resnet18", 10).to(gpu).train().load_from_pcmp(m)
    flat = FlatParams(m.parameters())
    opt = SGD(flat, lr=lr0, momentum=0.9, weight_decay=5e-5)
    topt = torch.optim.SGD(t.parameters(), lr=lr0, momentum=0.9, weight_decay=5e-5)
    lh, lt = [], []
    for i, (x, y) in enumerate(batches):
        lr = lr0 * min(1.0, (i + 1) / warm)
        opt.set_lr(lr)
        for gr in topt.param_groups:
            gr["lr"] = lr
        opt.zero_grad()
        loss = cross_entropy(m.forward_logits(x), y)
        loss.backward()
        opt.step()
        lh.append(loss.detach())
        topt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            tl = torch.nn.functional.cross_entropy(t(x).float(), y)
        tl.backward()
        topt.step()
        lt.append(tl.detach())
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det
    lh = torch.stack(lh).float().cpu()
    lt = torch.stack(lt).float().cpu()
    first_h, last_h = lh[:10].mean().item(), lh[-20:].mean().item()
    first_t, last_t = lt[:10].mean().item(), lt[-20:].mean().item()
    print(f"resnet18 convergence: hip {first_h:.3f} -> {last_h:.3f}; autocast {first_t:.3f} -> {last_t:.3f}")
    assert last_h < 0.5 * first_h and last_t < 0.5 * first_t
    assert abs(last_h - last_t) < 0.15 + 0.25 * max(last_h, last_t), (last_h, last_t)


def test_transfer_learning_flow_reaches_reference_accuracy(gpu):
    """The reference fine-tunes an ImageNet-pretrained backbone (nb :389, weights downloaded,
    :397-410); no download is possible here, so a short full-network 'pretraining' on a disjoint
    index range of the synthetic Imagenette-shaped set stands in for it.  Then the TL flow proper:
    freeze the backbone (BN stays in train mode, C2), new MLP head, NLL, Adam 3e-3, ONE epoch with
    per-epoch eval (the notebook's recipe, nb :436-446,:655-702) -- test accuracy >= 0.9 (P2 0.979)."""
    from pcmp.data.synthetic import BatchLoader, SyntheticImages
    from pcmp.engine.trainer import make_state, train_image_classifier
    from pcmp.models.layers import MLPHead
    from pcmp.models.resnet import resnet50
    res, B = 96, 64
    ds = SyntheticImages(28160, 10, res, seed=42, device=gpu)
    # "pretraining": 400 SGD steps over images 2560.. (never seen by the TL split below).  160 steps
    # left the frozen features on the edge: test accuracy 0.65-1.0 depending on which autotuned
    # kernel plans (and so which rounding) earlier tests had cached.
    torch.manual_seed(0)
    m = resnet50(num_classes=10).to(gpu).train()
    pre = make_state(m, "sgd", lr=0.05, momentum=0.9, weight_decay=5e-5)
    for i in range(400):
        pre.opt.set_lr(0.05 * min(1.0, (i + 1) / 30))
        x, y = ds.get_batch(list(range(2560 + i * B, 2560 + (i + 1) * B)))
        pre.zero_grad()
        pre.backward_step(cross_entropy(m.forward_logits(x), y))
    # transfer learning on images 0..2559: 80/20 split, 1 epoch
    m.freeze_backbone().replace_head(MLPHead(m.feature_dim, 512, 10, 0.2).to(gpu))
    idx = torch.randperm(2560, generator=torch.Generator().manual_seed(42)).tolist()
    split = int(0.2 * 2560)
    tr = BatchLoader(ds, B, device=gpu, indices=idx[split:], shuffle=True)
    te = BatchLoader(ds, B, device=gpu, indices=idx[:split], shuffle=True)
    state = make_state(m, "adam", lr=0.003)
    assert all(not p.requires_grad for n, p in m.named_parameters() if not n.startswith("fc."))
    lines = []
    train_image_classifier(state, tr, te, epochs=1, print_every=1, printer=lines.append)
    acc = state.history["test_acc"][-1]
    print("TL flow:", [l for l in lines if isinstance(l, str) and l.startswith("Epoch")])
    assert acc >= 0.9, state.history
