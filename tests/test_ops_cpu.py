"""CPU tests of the reference op layer, the dispatcher, FastDiv, RNG and the host parts."""
import pytest
import torch

import pcmp
from pcmp.ops import K, _lib, ref


def test_dispatch_cpu_uses_reference():
    x = torch.randn(2, 5, 5, 8)
    w = torch.randn(16, 3, 3, 8)
    y = K.conv_fwd(x, w, 1, 1, None, None, True, False)[0]
    yr = torch.relu(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), padding=1)).permute(0, 2, 3, 1)
    assert torch.allclose(y, yr, atol=1e-5)


def test_native_library_builds_and_registers_ops():
    assert _lib.LIB_PATH.exists(), "run __graft_entry__.build() first"
    assert _lib.load(), _lib.load_error()
    for name in ("conv_fwd", "conv_dgrad", "conv_wgrad", "bn_finalize", "lstm_seq_fwd", "attention_fwd",
                 "sgd_flat", "adam_flat", "text_encode", "layernorm_fwd", "embedding_fwd"):
        assert hasattr(torch.ops.pcmp, name), name


def test_gpu_tensor_without_native_raises(monkeypatch):
    class FakeT:
        is_cuda = True
    monkeypatch.setattr(_lib, "_loaded", False)
    monkeypatch.setattr(_lib, "LIB_PATH", _lib.LIB_PATH.parent / "missing.so")
    monkeypatch.setattr(_lib, "_backend", "hip")
    with pytest.raises(RuntimeError, match="Refusing to fall back"):
        _lib.use_native(FakeT())


def _fastdiv(d):
    s = 0
    while (1 << s) < d:
        s += 1
    m = ((1 << 32) * ((1 << s) - d)) // d + 1
    return m & 0xFFFFFFFF, s


@pytest.mark.parametrize("d", [1, 2, 3, 7, 14, 28, 49, 56, 112, 196, 784, 3136, 12544, 50176])
def test_fastdiv_formula(d):
    m, s = _fastdiv(d)
    import random
    vals = [0, 1, d - 1, d, d + 1, 2 ** 31 - 1] + [random.randrange(0, 2 ** 31) for _ in range(2000)]
    for n in vals:
        t = (n * m) >> 32
        assert (t + n) >> s == n // d, (n, d)


def test_hash_rng_uniform():
    u = ref.hash_uniform(123, torch.arange(100000))
    assert 0.49 < u.mean().item() < 0.51 and u.min() >= 0 and u.max() < 1
    assert torch.equal(u, ref.hash_uniform(123, torch.arange(100000)))
    assert not torch.equal(u, ref.hash_uniform(124, torch.arange(100000)))


def test_bn_reference_roundtrip_vs_autograd():
    torch.manual_seed(0)
    x = torch.randn(64, 16) * 3 + 1
    g, b = torch.rand(16) + 0.5, torch.randn(16)
    part = ref.bn_partials(x)
    mean, invstd, sc, sh = ref.bn_finalize(part, 64, g, b, None, None, 0.1, 1e-5)
    y = ref.bn_apply(x, sc, sh, None, None, None, True)
    xt = x.clone().requires_grad_(True)
    gt, bt = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yt = torch.relu(torch.nn.functional.batch_norm(xt, None, None, gt, bt, True, 0.1, 1e-5))
    assert torch.allclose(y, yt, atol=1e-5)
    dy = torch.randn_like(x)
    yt.backward(dy)
    p = ref.bn_bwd_reduce(dy, y, x, mean, invstd)[0]
    dg, db = torch.zeros(16), torch.zeros(16)
    coef = ref.bn_bwd_finalize(p, 64, g, mean, invstd, dg, db, False)
    dx = ref.bn_bwd_apply(dy, y, x, coef)[0]
    assert torch.allclose(dx, xt.grad, atol=1e-5)
    assert torch.allclose(dg, gt.grad, atol=1e-4) and torch.allclose(db, bt.grad, atol=1e-4)


def test_maxpool_reference_idx_roundtrip():
    x = torch.randn(2, 9, 9, 8)
    y, idx = ref.maxpool_fwd(x, 3, 2, 1, True)
    xt = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yt = torch.nn.functional.max_pool2d(xt, 3, 2, 1)
    dy = torch.randn_like(y)
    yt.backward(dy.permute(0, 3, 1, 2))
    assert torch.allclose(ref.maxpool_bwd(dy, idx, 9, 9, 3, 2, 1), xt.grad.permute(0, 2, 3, 1), atol=1e-6)


def test_batched_weight_transpose_reference():
    from pcmp.ops.params import compute_weight, compute_weight_t
    from pcmp.utils.flat import FlatParams
    ps = [torch.nn.Parameter(torch.randn(*s)) for s in [(16, 3, 3, 8), (32, 1, 1, 16), (8, 7, 7, 8)]]
    FlatParams(ps)
    for p in ps:
        wt = compute_weight_t(p, torch.bfloat16)
        assert wt.shape == (p.shape[3], p.shape[1], p.shape[2], p.shape[0])
        assert torch.equal(wt, compute_weight(p, torch.bfloat16).permute(3, 1, 2, 0))
    dy = torch.randn(2, 5, 5, 16).to(torch.bfloat16)
    w = compute_weight(ps[0], torch.bfloat16)
    assert torch.equal(K.conv_dgrad(dy, w, 5, 5, 1, 1, None, compute_weight_t(ps[0], torch.bfloat16)),
                       K.conv_dgrad(dy, w, 5, 5, 1, 1, None))


def test_mask_bits_roundtrip_reference():
    y = torch.randn(3, 5, 16).relu().to(torch.bfloat16)
    bits = ref.pack_mask_bits(y)
    assert bits.dtype == torch.uint8 and bits.numel() == y.numel() // 8
    assert torch.equal(ref.unpack_mask_bits(bits, y.shape) > 0, y.float() > 0)
    mb = torch.empty_like(bits)
    x = torch.randn(3, 5, 16).to(torch.bfloat16)
    sc, sh = torch.randn(16), torch.randn(16)
    out = ref.bn_apply(x, sc, sh, None, None, None, True, mb)
    assert torch.equal(mb, ref.pack_mask_bits(out))


@pytest.mark.parametrize("hw", [20, 21])
def test_stem_space_to_depth_equivalence(hw):
    """7x7/2 pad-3 conv == 4x4/1 unpadded conv over the 2x2 space-to-depth image with the filter
    embedded in 8x8 (the GPU stem); the filter / input gradients map back exactly."""
    from pcmp.ops.conv_blocks import s2d_input_grad, s2d_weight, s2d_weight_grad
    torch.manual_seed(0)
    x = torch.randn(2, 3, hw, hw).bfloat16().float()          # bf16-exact: the s2d image is bf16
    w = torch.zeros(5, 7, 7, 8)
    w[..., :3] = torch.randn(5, 7, 7, 3)
    y7 = torch.nn.functional.conv2d(x, w.permute(0, 3, 1, 2)[:, :3], stride=2, padding=3)
    xs = ref.image_to_s2d(x, 3, 1.0, None, None, False).float()
    assert xs.shape == (2, (hw + 7) // 2, (hw + 7) // 2, 16)
    xs_nhwc = ref.image_to_s2d(torch.nn.functional.pad(x.permute(0, 2, 3, 1), (0, 5)).bfloat16(), 3, 1.0, None,
                               None, True).float()
    assert torch.equal(xs, xs_nhwc)
    w4 = s2d_weight(w).requires_grad_(True)
    xs_ = xs.permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    y4 = torch.nn.functional.conv2d(xs_, w4.permute(0, 3, 1, 2))
    assert y4.shape == y7.shape
    torch.testing.assert_close(y4, y7, rtol=1e-5, atol=1e-4)
    # gradients: through the s2d conv, mapped back, equal the direct conv's
    dy = torch.randn_like(y7)
    y4.backward(dy)
    w7 = w.clone().requires_grad_(True)
    x7 = torch.nn.functional.pad(x.permute(0, 2, 3, 1), (0, 5)).contiguous().requires_grad_(True)
    torch.nn.functional.conv2d(x7.permute(0, 3, 1, 2), w7.permute(0, 3, 1, 2), stride=2, padding=3).backward(dy)
    torch.testing.assert_close(s2d_weight_grad(w4.grad), w7.grad[..., :4], rtol=1e-4, atol=1e-3)
    gx = s2d_input_grad(xs_.grad.permute(0, 2, 3, 1), hw, hw, 3, 8)
    torch.testing.assert_close(gx[..., :3], x7.grad[..., :3], rtol=1e-4, atol=1e-3)


def test_hash_rng_consecutive_calls_uncorrelated():
    """Eager dropout draws call k's mask at offset k << 32 (ops/functions.py).  The round-4 hash folded
    both index words into one lowbias32 round, so call k+1's values were an index permutation of call
    k's (advisor finding); the two-round hash must give independent streams: equal sorted values would
    expose a permutation, and the values of the same index must be uncorrelated."""
    n = 1 << 18
    idx = torch.arange(n, dtype=torch.int64)
    for k in (1, 77, 12345):
        u1 = ref.hash_uniform(1234, idx + (k << 32))
        u2 = ref.hash_uniform(1234, idx + ((k + 1) << 32))
        assert not torch.equal(torch.sort(u1).values, torch.sort(u2).values)
        c = torch.corrcoef(torch.stack([u1.double(), u2.double()]))[0, 1].item()
        assert abs(c) < 0.01, c
        m1, m2 = u1 >= 0.1, u2 >= 0.1
        both = (m1 & m2).double().mean().item()
        assert abs(both - 0.81) < 0.005, both
