"""igemm_dma32_kernel (round 5: one-barrier 32x32x16 LDS-DMA main loop + register-reduced epilogue)
against the fp32 PyTorch reference (ops/ref.py) and against the igemm_dma_kernel it replaces
(knob dma32 = 0), on grids large enough for the 4-wave LDS-DMA path (>= 256 tiles of 128x128, >= 3
K-tiles, source channels a multiple of 64): every FWD / DGRAD epilogue the conv paths use --
BN statistics, bias + residual + ReLU, stride-2 sub-pixel DGRAD rows, the fused BN-backward
reduction with tensor / bit / recomputed masks, the dual-BN form and the sub-sampled residual.
Reference shapes: SURVEY.md §2.4.1 (ResNet-50 conv layers, pytorch_training_inference_on_image.ipynb:454-635).
"""
import pytest
import torch

import pcmp  # noqa: F401
from pcmp.ops import ref

pytestmark = pytest.mark.gpu


def _ops():
    return torch.ops.pcmp


def rnd(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def close_el(a, b, rel=1e-2, abs_frac=5e-3):
    a, b = a.float(), b.float()
    lim = rel * b.abs() + abs_frac * b.abs().max()
    nbad = int(((a - b).abs() > lim).sum().item())
    assert nbad == 0, f"{nbad} elements outside the element-wise bound"


def close_sum(a, b, rtol=2e-2, atol=1.0):
    torch.testing.assert_close(a.double().sum(0), b.double().sum(0), rtol=rtol, atol=atol)


def both(fn):
    """fn() with the new kernel (dma32=1; dma32_modes=3 and dma32_dgrad_mink=1 also route the DGRADs
    the default policy keeps on the old kernel) and with the round-4 kernel (dma32=0)."""
    ops = _ops()
    old = ops.set_knob("dma32", 1)
    oldk = ops.set_knob("dma32_dgrad_mink", 1)
    oldm = ops.set_knob("dma32_modes", 3)
    try:
        a = fn()
        ops.set_knob("dma32", 0)
        b = fn()
    finally:
        ops.set_knob("dma32", old)
        ops.set_knob("dma32_dgrad_mink", oldk)
        ops.set_knob("dma32_modes", oldm)
    return a, b


SHAPES = [
    # N, H, W, C, K, R, stride, pad
    (20, 56, 56, 256, 64, 1, 1, 0),     # 128x64 tiles, 4 K-tiles (FWD); DGRAD 1 K-tile stays off
    (48, 28, 28, 64, 64, 3, 1, 1),      # 3x3 narrow: 128x64 tiles, 9 K-tiles
    (33, 28, 28, 64, 192, 3, 1, 1),     # gn = 192 (half-empty second tile column), M tail (25872 rows)
    (40, 28, 28, 128, 128, 3, 2, 1),    # stride-2 3x3: DGRAD sub-pixel classes
    (64, 28, 28, 256, 512, 1, 2, 0),    # 1x1 stride-2 downsample
    (64, 14, 14, 512, 512, 3, 1, 1),    # layer-4-like 3x3, 72 K-tiles
    (128, 14, 14, 1024, 256, 1, 1, 0),  # long-K 1x1 (16 K-tiles), DGRAD 4 K-tiles at gn = 1024
]


@pytest.mark.parametrize("shape", SHAPES)
def test_dma32_fwd(gpu, shape):
    torch.manual_seed(1)
    N, H, W, C, K, R, s, p = shape
    ops = _ops()
    x = rnd(N, H, W, C, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
    (y, st), (yo, sto) = both(lambda: ops.conv_fwd(x, w, s, p, None, None, False, True))
    yr, str_ = ref.conv_fwd(x, w, s, p, None, None, False, True)
    close_el(y, yr)
    close_el(y, yo)
    close_sum(st, str_)
    close_sum(st, sto, rtol=2e-3, atol=5e-1)
    bias = torch.randn(K, device=gpu)
    res = rnd(*yr.shape, dev=gpu)
    y2, y2o = both(lambda: ops.conv_fwd(x, w, s, p, bias, res, True, False)[0])
    y2r = ref.conv_fwd(x, w, s, p, bias, res, True, False)[0]
    close_el(y2, y2r)
    close_el(y2, y2o)
    assert (y2 >= 0).all()
    # deterministic: a second launch is bitwise equal
    y3, _ = both(lambda: ops.conv_fwd(x, w, s, p, bias, res, True, False)[0])
    assert torch.equal(y2, y3)


@pytest.mark.parametrize("shape", [
    (16, 14, 14, 256, 256, 3, 1, 1),    # layer-3 3x3 at B=16: 25 x 2 tiles of 128x128
    (64, 7, 7, 512, 512, 3, 1, 1),      # layer-4 3x3 at B=64: 25 x 4 tiles
    (9, 14, 14, 1024, 192, 1, 1, 0),    # 1x1, M tail, half-empty last 64-column tile
])
def test_small_grid_fwd_128x64(gpu, shape):
    """dma4_small_n64: FWD grids of fewer 128x128 tiles than CUs on 128x64 LDS-DMA tiles (every
    N tile writes its own columns of the per-M-tile BN partial rows) against fp32 PyTorch and the
    128x128 tiles."""
    torch.manual_seed(2)
    N, H, W, C, K, R, s, p = shape
    ops = _ops()
    x = rnd(N, H, W, C, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
    old = ops.set_knob("dma4_small_n64", 1)
    try:
        y, st = ops.conv_fwd(x, w, s, p, None, None, False, True)
        ops.set_knob("dma4_small_n64", 0)
        yo, sto = ops.conv_fwd(x, w, s, p, None, None, False, True)
    finally:
        ops.set_knob("dma4_small_n64", old)
    yr, str_ = ref.conv_fwd(x, w, s, p, None, None, False, True)
    close_el(y, yr)
    close_el(y, yo)
    close_sum(st, str_)
    close_sum(st, sto, rtol=2e-3, atol=5e-1)


@pytest.mark.parametrize("shape", SHAPES)
def test_dma32_dgrad(gpu, shape):
    torch.manual_seed(2)
    N, H, W, C, K, R, s, p = shape
    ops = _ops()
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    dy = rnd(N, P, Q, K, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * K)) ** 0.5)
    res = rnd(N, H, W, C, dev=gpu)
    dx, dxo = both(lambda: ops.conv_dgrad(dy, w, H, W, s, p, res.clone()))
    dxr = ref.conv_dgrad(dy, w, H, W, s, p, res)
    close_el(dx, dxr)
    close_el(dx, dxo)
    if R == 1 and s == 2:
        return   # a 1x1 stride-2 DGRAD leaves pixel classes uncovered: no fused BN-backward form
    xb = rnd(N, H, W, C, dev=gpu)
    mean, istd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    ymask = rnd(N, H, W, C, dev=gpu).relu()
    bits = ref.pack_mask_bits(ymask)
    # tail form: residual gradient + tensor mask, and the same with the mask as bits (bitwise equal)
    a, ao = both(lambda: ops.conv_dgrad_bnr(dy, w, H, W, s, p, res.clone(), ymask, xb, mean, istd,
                                            None, None, None, None, None))
    ar = ref.conv_dgrad_bnr(dy, w, H, W, s, p, res, ymask, xb, mean, istd, None, None, None)
    close_el(a[0], ar[0])
    close_el(a[0], ao[0])
    assert (a[0][ymask <= 0] == 0).all()
    close_sum(a[1], ar[1])
    close_sum(a[1], ao[1], rtol=2e-3, atol=5e-1)
    bits_form = lambda: ops.conv_dgrad_bnr(dy, w, H, W, s, p, res.clone(), None, xb, mean, istd,  # noqa: E731
                                           None, None, None, None, None, None, bits)
    old_stream = ops.set_knob("bnr_stream", 0)   # the bit-mask form of THIS kernel: bitwise equal
    try:
        ab, _ = both(bits_form)
    finally:
        ops.set_knob("bnr_stream", old_stream)
    for u, v in zip(ab, a):
        assert torch.equal(u, v)
    # with the default policy a short-K 1x1 bit-mask DGRAD may route to the streaming kernel
    # (bnr_stream.h: its own partial-row layout), so only values and column sums must agree
    ad = bits_form()
    close_el(ad[0], ar[0])
    close_sum(ad[1], ar[1])
    # intermediate form: mask recomputed from x
    sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
    m, mo = both(lambda: ops.conv_dgrad_bnr(dy, w, H, W, s, p, None, None, xb, mean, istd, None, None, None, sc, sh))
    mr = ref.conv_dgrad_bnr(dy, w, H, W, s, p, None, None, xb, mean, istd, None, None, None, sc, sh)
    close_el(m[0], mr[0])
    close_el(m[0], mo[0])
    assert ((m[0] == 0) | ((xb.float() * sc + sh) > 0)).all()
    close_sum(m[1], mr[1])
    if s == 1:
        # dual BN-reduce form (block input gradient into bn3 of the previous block + its downsample BN)
        x2 = rnd(N, H, W, C, dev=gpu)
        mean2, istd2 = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
        d, do = both(lambda: ops.conv_dgrad_bnr(dy, w, H, W, s, p, res.clone(), None, xb, mean, istd, x2, mean2, istd2,
                                                None, None, None, bits))
        dr = ref.conv_dgrad_bnr(dy, w, H, W, s, p, res, ymask, xb, mean, istd, x2, mean2, istd2)
        assert len(d) == 3
        close_el(d[0], dr[0])
        close_el(d[0], do[0])
        for u, v, uo in zip(d[1:], dr[1:], do[1:]):
            close_sum(u, v)
            close_sum(u, uo, rtol=2e-3, atol=5e-1)


def test_dma32_dgrad_sub_sampled_residual(gpu):
    """resid_sub on the new kernel: the compact half-resolution residual == its dense expansion, bitwise."""
    torch.manual_seed(3)
    ops = _ops()
    N, H, C, K, Kd = 64, 28, 256, 256, 512
    dh = rnd(N, H, H, K, dev=gpu)
    w = rnd(K, 3, 3, C, dev=gpu, scale=0.05)
    t_sub = ops.conv_dgrad(rnd(N, H // 2, H // 2, Kd, dev=gpu), rnd(Kd, 1, 1, C, dev=gpu, scale=0.05),
                           H // 2, H // 2, 1, 0, None)
    t_dense = ref.expand_sub_resid(t_sub, H, H)
    x = rnd(N, H, H, C, dev=gpu)
    mean, istd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    ymask = rnd(N, H, H, C, dev=gpu).relu()
    a = ops.conv_dgrad_bnr(dh, w, H, H, 1, 1, t_dense, ymask, x, mean, istd, None, None, None, None, None)
    b = ops.conv_dgrad_bnr(dh, w, H, H, 1, 1, t_sub, ymask, x, mean, istd, None, None, None, None, None, None, None,
                           None, None, True)
    for ta, tb in zip(a, b):
        assert torch.equal(ta, tb)
    r = ref.conv_dgrad_bnr(dh, w, H, H, 1, 1, t_sub, ymask, x, mean, istd, None, None, None, resid_sub=True)
    close_el(b[0], r[0])
