"""Numerics of every HIP kernel against the PyTorch fp32 reference of the same op (GPU only).

Inputs are bf16 (what the kernels consume); the reference computes in fp32 from the same bf16
values, so differences are accumulation order + output rounding.  Shapes cover the classes of
SURVEY.md §2.4.1 (stem 7x7/2 with Cin padded to 8, 1x1, 3x3, strided 3x3 and 1x1 downsample,
narrow and wide Cout, small-M linear).
"""
import pytest
import torch

import pcmp  # noqa: F401
from pcmp.ops import ref

pytestmark = pytest.mark.gpu


def _ops():
    return torch.ops.pcmp


def rnd(*shape, dev, scale=1.0, dtype=torch.bfloat16):
    return (torch.randn(*shape, device=dev) * scale).to(dtype)


def close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"max err {err} > {lim}"


def close_el(a, b, rel=1e-2, abs_frac=5e-3):
    """Element-wise bound |a - b| <= rel*|b| + abs_frac*max|b|: a localised error (one wrong tile,
    one wrong channel) fails even when it is small against the tensor's maximum."""
    a, b = a.float(), b.float()
    lim = rel * b.abs() + abs_frac * b.abs().max()
    bad = ((a - b).abs() > lim)
    nbad = int(bad.sum().item())
    assert nbad == 0, f"{nbad} elements outside the element-wise bound (worst {((a - b).abs() - lim).max().item():.3g})"


CONV_SHAPES = [
    # N, H, W, C, K, R, stride, pad
    (2, 32, 32, 8, 64, 7, 2, 3),      # stem (Cin padded 3->8)
    (2, 14, 14, 64, 64, 1, 1, 0),     # 1x1
    (2, 14, 14, 64, 256, 1, 1, 0),    # 1x1 expand
    (2, 14, 14, 64, 64, 3, 1, 1),     # 3x3
    (2, 14, 14, 128, 128, 3, 2, 1),   # 3x3 stride 2
    (2, 14, 14, 256, 512, 1, 2, 0),   # 1x1 stride-2 downsample
    (3, 7, 7, 512, 512, 3, 1, 1),     # layer4 3x3 (M not a multiple of the tile)
    (2, 14, 14, 24, 136, 3, 1, 1),    # channel counts off the tile grid (WGRAD gn = 216, gm = 136)
    (1, 7, 7, 512, 2048, 1, 1, 0),    # batch-1 inference: split-K forward
    (1, 14, 14, 256, 256, 3, 1, 1),   # batch-1 inference 3x3: split-K forward
    (5, 1, 1, 2048, 16, 1, 1, 0),     # linear, tiny M, N
    (64, 1, 1, 512, 1000 + 8, 1, 1, 0),  # linear 1000(+pad) classes
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd(gpu, shape):
    N, H, W, C, K, R, s, p = shape
    x = rnd(N, H, W, C, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
    bias = torch.randn(K, device=gpu)
    y, st = _ops().conv_fwd(x, w, s, p, None, None, False, True)
    yr, str_ = ref.conv_fwd(x, w, s, p, None, None, False, True)
    close(y, yr)
    close_el(y, yr)
    close(st.sum(0), str_.sum(0), rtol=2e-2, atol=1e-1)
    # fused bias + residual + relu epilogue
    res = rnd(*yr.shape, dev=gpu)
    y2 = _ops().conv_fwd(x, w, s, p, bias, res, True, False)[0]
    y2r = ref.conv_fwd(x, w, s, p, bias, res, True, False)[0]
    close(y2, y2r)


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_dgrad(gpu, shape):
    N, H, W, C, K, R, s, p = shape
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    dy = rnd(N, P, Q, K, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * K)) ** 0.5)
    dx = _ops().conv_dgrad(dy, w, H, W, s, p, None)
    dxr = ref.conv_dgrad(dy, w, H, W, s, p, None)
    close(dx, dxr)
    res = rnd(N, H, W, C, dev=gpu)
    # the native op may consume (reuse in place) the residual buffer for stride 2
    close(_ops().conv_dgrad(dy, w, H, W, s, p, res.clone()), ref.conv_dgrad(dy, w, H, W, s, p, res))


BNR_SHAPES = [
    # N, H, W, C, K, R, stride, pad, dual, resid
    (4, 14, 14, 64, 64, 3, 1, 1, False, False),     # bottleneck conv2 -> bn1
    (4, 14, 14, 64, 256, 1, 1, 0, False, False),    # conv3 -> bn2
    (4, 14, 14, 128, 128, 3, 2, 1, False, False),   # strided conv2 (sub-pixel classes) -> bn1
    (3, 7, 7, 256, 64, 1, 1, 0, True, True),        # block input grad -> previous bn3 + downsample bn
    (2, 9, 9, 64, 32, 3, 1, 1, False, True),        # M not a multiple of the tile, narrow K
]


@pytest.mark.parametrize("shape", BNR_SHAPES)
def test_conv_dgrad_bn_reduce_fused(gpu, shape):
    N, H, W, C, K, R, s, p, dual, has_res = shape
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    dy = rnd(N, P, Q, K, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * K)) ** 0.5)
    ymask = rnd(N, H, W, C, dev=gpu).relu()
    x = rnd(N, H, W, C, dev=gpu)
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    x2 = rnd(N, H, W, C, dev=gpu) if dual else None
    mean2, invstd2 = (torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5) if dual else (None, None)
    res = rnd(N, H, W, C, dev=gpu) if has_res else None
    out = _ops().conv_dgrad_bnr(dy, w, H, W, s, p, res.clone() if has_res else None, ymask, x, mean, invstd,
                                x2, mean2, invstd2, None, None)
    outr = ref.conv_dgrad_bnr(dy, w, H, W, s, p, res, ymask, x, mean, invstd, x2, mean2, invstd2)
    assert len(out) == len(outr) == (3 if dual else 2)
    close(out[0], outr[0])
    assert (out[0][ymask <= 0] == 0).all()
    for a, b in zip(out[1:], outr[1:]):
        close(a.sum(0), b.sum(0), rtol=2e-2, atol=2e-1)
    # block-output form: the mask as bits (bn_apply mbits) gives exactly the tensor-mask result
    bits = ref.pack_mask_bits(ymask)
    outb = _ops().conv_dgrad_bnr(dy, w, H, W, s, p, res.clone() if has_res else None, None, x, mean, invstd,
                                 x2, mean2, invstd2, None, None, None, bits)
    for a, b in zip(outb, out):
        assert torch.equal(a, b)
    if not dual:
        # intermediate-layer form: ReLU mask recomputed from x (relu(x * scale + shift) > 0)
        sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
        out = _ops().conv_dgrad_bnr(dy, w, H, W, s, p, res.clone() if has_res else None, None, x, mean, invstd,
                                    None, None, None, sc, sh)
        outr = ref.conv_dgrad_bnr(dy, w, H, W, s, p, res, None, x, mean, invstd, None, None, None, sc, sh)
        close(out[0], outr[0])
        assert ((out[0] == 0) | ((x.float() * sc + sh) > 0)).all()
        close(out[1].sum(0), outr[1].sum(0), rtol=2e-2, atol=2e-1)


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_wgrad(gpu, shape):
    N, H, W, C, K, R, s, p = shape
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    dy = rnd(N, P, Q, K, dev=gpu)
    x = rnd(N, H, W, C, dev=gpu)
    out = torch.empty(K, R, R, C, device=gpu)
    outr = torch.empty_like(out)
    _ops().conv_wgrad(dy, x, out, R, R, s, p, False)
    ref.conv_wgrad(dy, x, outr, R, R, s, p, False)
    close(out, outr, rtol=1e-2, atol=1e-2)
    _ops().conv_wgrad(dy, x, out, R, R, s, p, True)
    close(out, 2 * outr, rtol=1e-2, atol=2e-2)


def test_conv_wgrad_large_k_splitk(gpu):
    # reduction over N*P*Q = 32*28*28 = 25088 rows -> split-K path
    x = rnd(32, 28, 28, 128, dev=gpu)
    dy = rnd(32, 28, 28, 128, dev=gpu)
    out = torch.empty(128, 3, 3, 128, device=gpu)
    outr = torch.empty_like(out)
    _ops().conv_wgrad(dy, x, out, 3, 3, 1, 1, False)
    ref.conv_wgrad(dy, x, outr, 3, 3, 1, 1, False)
    close(out, outr, rtol=1e-2, atol=1e-1)


@pytest.mark.parametrize("C", [8, 64, 256, 2048])
def test_bn_forward_backward(gpu, C):
    M = 3000
    x = rnd(M, C, dev=gpu) * 2 + 0.5
    x2 = rnd(M, C, dev=gpu)
    g = torch.rand(C, device=gpu) + 0.5
    b = torch.randn(C, device=gpu)
    rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    rm2, rv2 = rm.clone(), rv.clone()
    part = _ops().bn_partials(x)
    partr = ref.bn_partials(x)
    close(part.sum(0), partr.sum(0), rtol=1e-3, atol=1e-1)
    mean, invstd, sc, sh = _ops().bn_finalize(part, M, g, b, rm, rv, 0.1, 1e-5)
    meanr, invstdr, scr, shr = ref.bn_finalize(partr, M, g, b, rm2, rv2, 0.1, 1e-5)
    close(mean, meanr, 1e-4, 1e-4)
    close(invstd, invstdr, 1e-3, 1e-4)
    close(rm, rm2, 1e-4, 1e-5)
    close(rv, rv2, 1e-3, 1e-4)
    y = _ops().bn_apply(x, sc, sh, x2, None, None, True)
    yr = ref.bn_apply(x, scr, shr, x2, None, None, True)
    close(y, yr)
    mb = torch.empty(y.numel() // 8, dtype=torch.uint8, device=gpu)
    assert torch.equal(_ops().bn_apply(x, sc, sh, x2, None, None, True, mb), y)
    assert torch.equal(mb, ref.pack_mask_bits(y))
    dy = rnd(M, C, dev=gpu)
    p1 = _ops().bn_bwd_reduce(dy, y, x, mean, invstd, None, None, None)[0]
    # the ReLU mask comes from the kernel's own y on both sides: a bf16 rounding flip of y at 0 would
    # otherwise switch one element's gradient on or off (a mask disagreement, not a numerics error)
    p1r = ref.bn_bwd_reduce(dy, y, x, meanr, invstdr, None, None, None)[0]
    close(p1.sum(0), p1r.sum(0), 1e-2, 1e-1)
    dg, db = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
    dgr, dbr = torch.empty_like(dg), torch.empty_like(db)
    coef = _ops().bn_bwd_finalize(p1, M, g, mean, invstd, dg, db, False)
    coefr = ref.bn_bwd_finalize(p1r, M, g, meanr, invstdr, dgr, dbr, False)
    close(dg, dgr, 1e-2, 1e-1)
    close(db, dbr, 1e-2, 1e-1)
    dx, gg = _ops().bn_bwd_apply(dy, y, x, coef, None, None, True)
    dxr, ggr = ref.bn_bwd_apply(dy, y, x, coefr, None, None, True)
    close(dx, dxr)
    close(gg, ggr)


@pytest.mark.parametrize("T,C", [(65, 64), (392, 256), (512, 2048), (300, 72), (1568, 2048), (6272, 64), (14336, 64), (785, 136)])
def test_bn_wide_finalize(gpu, T, C):
    """One-launch finalize: the wide kernel (64 < T <= bn_wide_rows partial rows) == the two-stage
    path (bn_wide_rows = 64) to fp64 rounding; above bn_wide_rows the two-stage path runs; for the
    forward (mean / invstd / scale / shift / running stats) and backward (dgamma / dbeta / coef)
    finalize; against an fp64 torch reduction; repeated calls bitwise equal."""
    ops = _ops()
    g = torch.Generator(device=gpu).manual_seed(T + C)
    part = torch.randn(T, 2, C, device=gpu, generator=g)
    part[:, 1] = part[:, 1].abs() * 4 + 2          # sum of squares: positive, var > 0
    gam = torch.rand(C, device=gpu, generator=g) + 0.5
    bet = torch.randn(C, device=gpu, generator=g)
    mean, invstd = torch.randn(C, device=gpu, generator=g), torch.rand(C, device=gpu, generator=g) + 0.5
    count = T * 16
    outs = {}
    prev = ops.set_knob("bn_wide_rows", 512)
    try:
        # two-stage path, default path (twice)
        for v in (64, 512, 512):
            ops.set_knob("bn_wide_rows", v)
            rm, rv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
            fwd = ops.bn_finalize(part, count, gam, bet, rm, rv, 0.1, 1e-5)
            dg, db = torch.full((C,), 0.5, device=gpu), torch.full((C,), 0.25, device=gpu)
            coef = ops.bn_bwd_finalize(part, count, gam, mean, invstd, dg, db, True)
            outs.setdefault(v, []).append([t.clone() for t in (*fwd, rm, rv, dg, db, coef)])
    finally:
        ops.set_knob("bn_wide_rows", prev)
    base = outs[512][0]
    for a, b in zip(base, outs[512][1]):
        assert torch.equal(a, b)
    for a, b in zip(base, outs[64][0]):
        if T > 512:   # both the two-stage path
            assert torch.equal(a, b)
        else:
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)
    s = part.double().sum(0)
    m = s[0] / count
    var = (s[1] / count - m * m).clamp_min(0)
    close(base[0], m.float(), 1e-6, 1e-6)
    close(base[1], (1.0 / torch.sqrt(var + 1e-5)).float(), 1e-5, 1e-6)
    close(base[7], (0.25 + s[0]).float(), 1e-6, 1e-4)    # dbeta accumulated
    close(base[6], (0.5 + s[1]).float(), 1e-6, 1e-4)     # dgamma accumulated


def test_maxpool_gap(gpu):
    x = rnd(2, 17, 17, 64, dev=gpu)
    y, idx = _ops().maxpool_fwd(x, 3, 2, 1, True)
    yr, idxr = ref.maxpool_fwd(x, 3, 2, 1, True)
    close(y, yr, 0, 0)
    dy = rnd(*y.shape, dev=gpu)
    close(_ops().maxpool_bwd(dy, idx, 17, 17, 3, 2, 1), ref.maxpool_bwd(dy, idxr, 17, 17, 3, 2, 1))
    g = _ops().gap_fwd(x)
    close(g, ref.gap_fwd(x))
    dg = rnd(2, 64, dev=gpu)
    close(_ops().gap_bwd(dg, 17, 17), ref.gap_bwd(dg, 17, 17))


@pytest.mark.parametrize("V", [10, 2, 1000])
def test_softmax_xent(gpu, V):
    z = torch.randn(37, V, device=gpu)
    y = torch.randint(0, V, (37,), device=gpu)
    y[3] = -100
    r = _ops().softmax_xent(z, y, True, True, 0.5, -100)
    rr = ref.softmax_xent(z, y, True, True, 0.5, -100)
    for a, b in zip(r, rr):
        close(a, b, 1e-4, 1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_loss_mean_grad_scale_log_softmax_bwd(gpu, dtype):
    V = 10
    z = torch.randn(37, V, device=gpu).to(dtype)
    y = torch.randint(0, V, (37,), device=gpu)
    y[3] = -100
    y[5] = -100
    r = _ops().softmax_xent(z, y, True, True, 1.0, -100)
    lm = _ops().loss_mean(r[0], y, V, -100)
    lmr = ref.loss_mean(r[0], y, V, -100)
    close(lm, lmr, 1e-5, 1e-6)
    assert lm[1].item() == 35.0
    gout = torch.tensor([0.7], device=gpu)
    close(_ops().xent_grad_scale(r[2], gout, lm[1:2]), ref.xent_grad_scale(r[2], gout, lm[1:2]), 1e-2, 1e-6)
    # log-softmax backward against autograd of torch.log_softmax in fp32
    g = torch.randn(37, V, device=gpu).to(dtype)
    zf = z.float().requires_grad_(True)
    torch.log_softmax(zf, 1).backward(g.float())
    dz = _ops().log_softmax_bwd(g, r[1])
    assert dz.dtype == dtype
    close(dz, zf.grad, 1e-2 if dtype == torch.bfloat16 else 1e-5, 1e-6)


def test_dropout_matches_reference_rng(gpu):
    x = rnd(4096, dev=gpu)
    y = _ops().dropout(x, 0.2, 1234, 77 << 32)
    yr = ref.dropout(x, 0.2, 1234, 77 << 32)
    close(y, yr, 0, 1e-2)
    keep = (y != 0).float().mean().item()
    assert 0.75 < keep < 0.85


def test_optimizers(gpu):
    n = 4096 * 3
    w = torch.randn(n, device=gpu)
    g = torch.randn(n, device=gpu)
    lr = torch.tensor([0.1], device=gpu)
    gs = torch.tensor([0.5], device=gpu)
    for first in (True, False):
        w1, w2 = w.clone(), w.clone()
        m1, m2 = torch.randn(n, device=gpu), None
        m2 = m1.clone()
        s1 = torch.empty(n, device=gpu, dtype=torch.bfloat16)
        s2 = s1.clone()
        _ops().sgd_flat(w1, g, m1, s1, None, lr, gs, 0.9, 0.0, 1e-4, True, first)
        ref.sgd_flat(w2, g, m2, s2, None, lr, gs, 0.9, 0.0, 1e-4, True, first)
        close(w1, w2, 1e-5, 1e-6)
        close(m1, m2, 1e-5, 1e-6)
        close(s1, s2, 1e-2, 1e-2)
    step = torch.tensor([3.0], device=gpu)
    for dec in (False, True):
        w1, w2 = w.clone(), w.clone()
        a1, b1 = torch.randn(n, device=gpu), torch.rand(n, device=gpu)
        a2, b2 = a1.clone(), b1.clone()
        _ops().adam_flat(w1, g, a1, b1, None, None, lr, gs, step, 0.9, 0.999, 1e-8, 0.01, dec)
        ref.adam_flat(w2, g, a2, b2, None, None, lr, gs, step.cpu(), 0.9, 0.999, 1e-8, 0.01, dec)
        close(w1, w2, 1e-5, 1e-5)
    norm, coef = _ops().grad_clip_coef(g, 1.0, 1.0, 0.25)
    normr, coefr = ref.grad_clip_coef(g, 1.0, 1.0, 0.25)
    close(norm, normr, 1e-5, 1e-4)
    close(coef, coefr, 1e-5, 1e-7)
    # two-phase form (per-bucket partial sums, one coefficient): the same norm over uneven buckets
    cuts = [0, 4096, 4096 + 1024 * 5, n]
    nb = [ref.sumsq_blocks(cuts[i + 1] - cuts[i]) for i in range(3)]
    part = torch.full((sum(nb),), float("nan"), device=gpu)
    off = 0
    for i in range(3):
        _ops().grad_sumsq_parts(g[cuts[i]:cuts[i + 1]], part, off)
        off += nb[i]
    norm2, coef2 = _ops().clip_coef_parts(part, 1.0, 1.0, 0.25)
    close(norm2, normr, 1e-5, 1e-4)
    close(coef2, coefr, 1e-5, 1e-7)


def test_input_conversion(gpu):
    x = torch.rand(2, 3, 9, 11, device=gpu)
    close(_ops().nchw_to_nhwc(x, 8, 1.0, None, None), ref.nchw_to_nhwc(x, 8, 1.0), 0, 1e-2)
    xu = (torch.rand(2, 3, 9, 11, device=gpu) * 255).to(torch.uint8)
    close(_ops().nchw_to_nhwc(xu, 8, 1 / 255, None, None), ref.nchw_to_nhwc(xu, 8, 1 / 255), 0, 1e-2)


@pytest.mark.parametrize("M,C", [(4096, 768), (4096, 3072), (37, 24), (256, 1000 + 8), (1, 64)])
def test_colsum_bias_grad(gpu, M, C):
    x = rnd(M, C, dev=gpu)
    ref_sum = x.float().sum(0)
    out = torch.empty(C, device=gpu)
    _ops().colsum(x, out, False)
    close(out, ref_sum, rtol=1e-4, atol=1e-3)
    _ops().colsum(x, out, True)
    close(out, 2 * ref_sum, rtol=1e-4, atol=2e-3)


# Shapes large enough for the 8-wave LDS-DMA kernel (BM=256 tiles >= 240, >= 4 K-tiles)
BIG_SHAPES = [
    # N, H, W, C, K, R, stride, pad
    (20, 56, 56, 64, 256, 3, 1, 1),     # FWD BN=256 (gn=256)
    (20, 56, 56, 128, 128, 3, 1, 1),    # FWD/DGRAD BN=128
    (20, 112, 112, 64, 128, 3, 2, 1),   # strided FWD; sub-pixel DGRAD classes
    (20, 56, 56, 256, 64, 1, 1, 0),     # DGRAD gn=256 over K=64 x 1x1 -> 1 K-tile (old kernel) / FWD gk=256
    (20, 56, 56, 256, 64, 3, 1, 1),     # DGRAD gn=256, 9 K-tiles -> 8-wave kernel incl. BN-reduce epilogue
    (5, 56, 56, 256, 512, 3, 1, 1),     # M tail (15680 = 61.25 tiles), N = 2 x 256
    # ResNet-50 layer3 at B=256: 196 BM=256 tiles (the 8-wave kernel's lower grid bound)
    (256, 14, 14, 256, 256, 3, 1, 1),
    (256, 14, 14, 1024, 256, 1, 1, 0),
    (256, 28, 28, 256, 256, 3, 2, 1),   # layer3.0 conv2: stride-2 DGRAD parity classes of 196 tiles
    # narrow outputs over >= 131072 pixels: BM=256 x BN=64 tiles (4 waves along M)
    (48, 56, 56, 64, 64, 3, 1, 1),
    (48, 56, 56, 256, 64, 1, 1, 0),
    (12, 224, 224, 8, 64, 7, 2, 3),     # stem (FWD 7x7/2; DGRAD over 64 -> 8 channels stays 4-wave)
]


@pytest.mark.parametrize("shape", BIG_SHAPES)
def test_conv_large_shapes_8wave(gpu, shape):
    N, H, W, C, K, R, s, p = shape
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    x = rnd(N, H, W, C, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
    y, st = _ops().conv_fwd(x, w, s, p, None, None, False, True)
    yr, str_ = ref.conv_fwd(x, w, s, p, None, None, False, True)
    close(y, yr)
    close_el(y, yr)
    close(st.sum(0), str_.sum(0), rtol=2e-2, atol=5e-1)
    bias = torch.randn(K, device=gpu)
    res = rnd(*yr.shape, dev=gpu)
    close(_ops().conv_fwd(x, w, s, p, bias, res, True, False)[0], ref.conv_fwd(x, w, s, p, bias, res, True, False)[0])
    dy = rnd(N, P, Q, K, dev=gpu)
    wd = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * K)) ** 0.5)
    dres = rnd(N, H, W, C, dev=gpu)
    close(_ops().conv_dgrad(dy, wd, H, W, s, p, dres.clone()), ref.conv_dgrad(dy, wd, H, W, s, p, dres))
    # fused BN-backward reduction (intermediate form: mask from x, and tail form: mask tensor)
    xb = rnd(N, H, W, C, dev=gpu)
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
    out = _ops().conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)
    outr = ref.conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)
    close(out[0], outr[0])
    close(out[1].sum(0), outr[1].sum(0), rtol=2e-2, atol=1.0)
    ymask = rnd(N, H, W, C, dev=gpu).relu()
    out = _ops().conv_dgrad_bnr(dy, wd, H, W, s, p, dres.clone(), ymask, xb, mean, invstd, x, mean, invstd, None, None)
    outr = ref.conv_dgrad_bnr(dy, wd, H, W, s, p, dres, ymask, xb, mean, invstd, x, mean, invstd)
    close(out[0], outr[0])
    for a, b in zip(out[1:], outr[1:]):
        close(a.sum(0), b.sum(0), rtol=2e-2, atol=1.0)


def test_batched_weight_transpose_and_dgrad_with_pretransposed(gpu):
    """FlatParams' transposed conv-weight arena (one wt_transpose_multi launch) equals the per-call
    transpose, and DGRAD with the pre-transposed weight equals DGRAD without it."""
    from pcmp.ops.params import bump_weight_gen, compute_weight, compute_weight_t
    from pcmp.utils.flat import FlatParams
    shapes = [(64, 3, 3, 64), (256, 1, 1, 64), (72, 7, 7, 8), (512, 1, 1, 256), (128, 3, 3, 128)]
    ps = [torch.nn.Parameter(torch.randn(*s, device=gpu) * 0.05) for s in shapes]
    # channel counts off the 8-element grid take the kernel's 2-byte path (the rest its 16-byte path)
    odd = torch.nn.Parameter(torch.randn(20, 3, 3, 12, device=gpu) * 0.05)
    ps[2]._pcmp_s2_pad = 3     # stride-2 7x7 and 3x3 (ConvBN marks them): class-blocked layout
    ps[4]._pcmp_s2_pad = 1
    lin = torch.nn.Parameter(torch.randn(40, 24, device=gpu))     # 2-D: no transposed copy
    flat = FlatParams(ps + [odd, lin])
    assert getattr(lin, "_flat_owner", None) is None
    assert torch.equal(compute_weight_t(odd, torch.bfloat16),
                       compute_weight(odd, torch.bfloat16).permute(3, 1, 2, 0).contiguous())
    for p in ps:
        wt = compute_weight_t(p, torch.bfloat16)
        full = compute_weight(p, torch.bfloat16).permute(3, 1, 2, 0).contiguous()   # [C,R,S,K]
        pad = getattr(p, "_pcmp_s2_pad", None)
        if pad is None:
            assert torch.equal(wt, full)
            continue
        blocks = [full[:, (oph + pad) & 1::2, (opw + pad) & 1::2, :].reshape(-1) for oph in (0, 1) for opw in (0, 1)]
        assert wt.dim() == 1 and torch.equal(wt, torch.cat(blocks))
    # stale after a weight change -> refreshed on the next request
    flat.master.mul_(-1.0)
    flat.refresh_shadows()
    p = ps[0]
    assert torch.equal(compute_weight_t(p, torch.bfloat16), compute_weight(p, torch.bfloat16).permute(3, 1, 2, 0).contiguous())
    bump_weight_gen()
    # the class-blocked stride-2 weight feeds the fused DGRAD + BN-reduce path too
    p4 = ps[4]
    dy4 = rnd(2, 7, 7, 128, dev=gpu)
    x4 = rnd(2, 14, 14, 128, dev=gpu)
    mean4, istd4 = torch.randn(128, device=gpu) * 0.1, torch.rand(128, device=gpu) + 0.5
    sc4, sh4 = torch.rand(128, device=gpu) + 0.5, torch.randn(128, device=gpu) * 0.1
    w4 = compute_weight(p4, torch.bfloat16)
    r_a = _ops().conv_dgrad_bnr(dy4, w4, 14, 14, 2, 1, None, None, x4, mean4, istd4, None, None, None, sc4, sh4)
    r_b = _ops().conv_dgrad_bnr(dy4, w4, 14, 14, 2, 1, None, None, x4, mean4, istd4, None, None, None, sc4, sh4,
                                compute_weight_t(p4, torch.bfloat16))
    for ta, tb in zip(r_a, r_b):
        assert torch.equal(ta, tb)
    for (K_, R, S, C), p, (s, pad) in zip(shapes, ps, [(1, 1), (1, 0), (2, 3), (2, 0), (2, 1)]):
        N, H, W = 2, 14, 14
        P, Q = (H + 2 * pad - R) // s + 1, (W + 2 * pad - S) // s + 1
        dy = rnd(N, P, Q, K_, dev=gpu)
        w = compute_weight(p, torch.bfloat16)
        a = _ops().conv_dgrad(dy, w, H, W, s, pad, None)
        b = _ops().conv_dgrad(dy, w, H, W, s, pad, None, compute_weight_t(p, torch.bfloat16))
        assert torch.equal(a, b)


def test_stem_fused_bn_maxpool(gpu):
    """Fused stem: maxpool with the BN+ReLU prologue == bn_apply then maxpool (bit-exact values and
    argmax); fused backward == maxpool_bwd then the masked BN-backward reduction."""
    torch.manual_seed(3)
    N, H, W, C = 4, 28, 28, 64
    c = rnd(N, H, W, C, dev=gpu)
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.3
    a = _ops().bn_apply(c, sc, sh, None, None, None, True)
    y0, i0 = _ops().maxpool_fwd(a, 3, 2, 1, True)
    y1, i1 = _ops().maxpool_fwd(c, 3, 2, 1, True, sc, sh)
    assert torch.equal(y0, y1)
    assert torch.equal(i0, i1)
    dy = rnd(*y1.shape, dev=gpu)
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    g, part = _ops().maxpool_bwd_bnr(dy, i1, c, mean, invstd, sc, sh, 3, 2, 1)
    da = _ops().maxpool_bwd(dy, i1, H, W, 3, 2, 1)
    gr = torch.where(a.float() > 0, da.float(), torch.zeros_like(da.float())).to(torch.bfloat16)
    assert torch.equal(g, gr)
    pr = ref.bn_bwd_reduce(gr, None, c, mean, invstd)[0]
    close(part.sum(0), pr.sum(0), rtol=1e-3, atol=1e-2)
    gref, pref = ref.maxpool_bwd_bnr(dy, i1, c, mean, invstd, sc, sh, 3, 2, 1)
    close(g, gref)
    close(part.sum(0), pref.sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("H,W", [(28, 28), (17, 23), (112, 112)])
def test_pool3s2_specialised(gpu, H, W):
    """The specialised 3x3/s2/p1 stem pooling kernels (knob pool3s2) == the generic kernels, bitwise:
    plain and BN-prologue forward (values + argmax, with ties and a NaN), fused backward (g + partials)."""
    ops = _ops()
    torch.manual_seed(H * W)
    N, C = 2 if H > 100 else 3, 64
    c = rnd(N, H, W, C, dev=gpu)
    c[0, 1:3, 1:3, :8] = 0.5                  # ties inside a window
    c[1, 4, 5, 9] = float("nan")
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.3
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    res = {}
    prev_quad = ops.set_knob("pool_quad", 0)   # the 2x2-quad backward sums its partials in another order
    try:
        for v in (0, 1):
            ops.set_knob("pool3s2", v)
            y, i = ops.maxpool_fwd(c, 3, 2, 1, True)
            yb, ib = ops.maxpool_fwd(c, 3, 2, 1, True, sc, sh)
            dy = torch.Generator(device=gpu).manual_seed(7)
            dy = torch.randn(yb.shape, device=gpu, generator=dy).to(torch.bfloat16)
            g, part = ops.maxpool_bwd_bnr(dy, ib, c, mean, invstd, sc, sh, 3, 2, 1)
            res[v] = (y, i, yb, ib, g, part)
        ops.set_knob("pool_quad", 1)
        gq, partq = ops.maxpool_bwd_bnr(dy, ib, c, mean, invstd, sc, sh, 3, 2, 1)
    finally:
        ops.set_knob("pool3s2", 1)
        ops.set_knob("pool_quad", prev_quad)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b) or (a.is_floating_point() and torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0)))
    # the quad kernel (even H, W): g bitwise; the per-channel sums equal up to fp32 summation order
    g1, part1 = res[1][4], res[1][5]
    assert torch.equal(gq.nan_to_num(7.0), g1.nan_to_num(7.0))
    close(partq.sum(0).nan_to_num(0.0), part1.sum(0).nan_to_num(0.0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("src", ["f32", "u8", "nhwc", "nhwc_f32"])
def test_image_to_s2d(gpu, src):
    """Stem space-to-depth kernel == the PyTorch reference (NCHW f32 / u8 with scale, NHWC bf16, NHWC
    fp32 -> fp32 for the fp32 stem)."""
    torch.manual_seed(0)
    if src == "f32":
        x, scale, nhwc = torch.rand(3, 3, 37, 30, device=gpu), 1.0, False
    elif src == "u8":
        x, scale, nhwc = torch.randint(0, 256, (3, 3, 30, 37), device=gpu, dtype=torch.uint8), 1 / 255, False
    elif src == "nhwc_f32":
        x, scale, nhwc = torch.randn(3, 31, 36, 8, device=gpu), 1.0, True
    else:
        x, scale, nhwc = rnd(3, 31, 36, 8, dev=gpu), 1.0, True
    y = _ops().image_to_s2d(x, 3, scale, None, None, nhwc)
    yr = ref.image_to_s2d(x, 3, scale, None, None, nhwc)
    assert y.shape == yr.shape
    assert torch.equal(y, yr)
    if not nhwc:   # the fp32 stem's one-pass form: NCHW f32 / u8 -> fp32 space-to-depth image
        yf = _ops().image_to_s2d_f32(x, 3, scale)
        yfr = ref.image_to_s2d_f32(x, 3, scale)
        assert yf.dtype == torch.float32
        torch.testing.assert_close(yf, yfr, rtol=1e-6, atol=1e-7)


def test_splitk_fwd_repeated(gpu):
    """Batch-1 split-K FWD (fp32 partial slabs + reduction/epilogue pass): repeated launches of several
    shapes with and without bias / residual / ReLU; bitwise reproducible."""
    torch.manual_seed(0)
    for rep in range(3):
        for (H, C, K, R) in [(7, 512, 2048, 1), (14, 256, 256, 3), (7, 2048, 512, 1), (7, 512, 512, 3)]:
            p = R // 2
            x = rnd(1, H, H, C, dev=gpu)
            w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
            bias = torch.randn(K, device=gpu)
            res = rnd(1, H, H, K, dev=gpu) if rep != 1 else None
            relu = rep != 2
            y = _ops().conv_fwd(x, w, 1, p, bias, res, relu, False)[0]
            yr = ref.conv_fwd(x, w, 1, p, bias, res, relu, False)[0]
            close(y, yr)
            # bitwise reproducible (fixed split order)
            assert torch.equal(y, _ops().conv_fwd(x, w, 1, p, bias, res, relu, False)[0])


def test_planned_inference_convs_match_reference(gpu):
    """The autotuned small-M FWD plan (kernel tile x K-split, csrc/igemm.hip plan_gemm) on ResNet-50
    batch-1 shapes (incl. stride 2) matches the reference and the unplanned round-1 path."""
    torch.manual_seed(1)
    ops = _ops()
    shapes = [(56, 64, 64, 3, 1), (28, 128, 128, 3, 1), (56, 128, 128, 3, 2), (14, 1024, 256, 1, 1),
              (14, 256, 1024, 1, 1), (7, 512, 512, 3, 1), (14, 1024, 2048, 1, 2)]
    for (H, C, K, R, s) in shapes:
        p = R // 2
        x = rnd(1, H, H, C, dev=gpu)
        w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
        bias = torch.randn(K, device=gpu)
        yr = ref.conv_fwd(x, w, s, p, bias, None, True, False)[0]
        ops.set_knob("gemm_plan", 0)
        try:
            y0 = ops.conv_fwd(x, w, s, p, bias, None, True, False)[0]
        finally:
            ops.set_knob("gemm_plan", 1)
        y1 = ops.conv_fwd(x, w, s, p, bias, None, True, False)[0]
        close(y0, yr)
        close(y1, yr)
        assert torch.equal(y1, ops.conv_fwd(x, w, s, p, bias, None, True, False)[0])   # cached plan, fixed order
    plans = ops.gemm_plans()
    assert any("|1," in k for k in plans), plans   # batch-1 geometry keys were planned


@pytest.mark.parametrize("kind", [3, 4, 6])
def test_small_m_plan_kinds_match_reference(gpu, kind):
    """Each small-M candidate kernel (register 64x64 / 32x64, skinny register-direct) forced through
    the planner, with and without K-splits (the planner times 1..32 splits), vs the fp32 reference;
    bias + residual + ReLU epilogues, batch-1 layer-3/4 shapes incl. stride 2 and the classifier."""
    torch.manual_seed(2)
    ops = _ops()
    ops.set_knob("plan_force", kind)
    try:
        for (H, C, K, R, s, use_res) in [(14, 256, 256, 3, 1, False), (14, 256, 256, 3, 2, False),
                                         (7, 2048, 512, 1, 1, False), (7, 512, 2048, 1, 1, True),
                                         (1, 2048, 1000, 1, 1, False), (14, 1024, 256, 1, 1, False)]:
            p = R // 2
            x = rnd(1, H, H, C, dev=gpu)
            w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
            bias = torch.randn(K, device=gpu)
            Ho = (H + 2 * p - R) // s + 1
            res = rnd(1, Ho, Ho, K, dev=gpu) if use_res else None
            y = ops.conv_fwd(x, w, s, p, bias, res, True, False)[0]
            yr = ref.conv_fwd(x, w, s, p, bias, res, True, False)[0]
            close(y, yr)
    finally:
        ops.set_knob("plan_force", -1)


def test_dgrad_bnr2_kernel_variants(gpu):
    """Dual BN-reduce DGRAD (the DGRAD into a block tail with a downsample BN): the one-tile kernel at
    epilogue depth 2 (default) and at depth 4 give the same masked gradient bitwise and the same
    BN-backward sums."""
    torch.manual_seed(5)
    ops = _ops()
    N, H, C, K = 16, 28, 256, 64          # 12,544 rows: wide short-K GEMM (gk = 64, gn = 256)
    w = rnd(K, 1, 1, C, dev=gpu, scale=0.1)
    dy = rnd(N, H, H, K, dev=gpu)
    xb, x2, res = rnd(N, H, H, C, dev=gpu), rnd(N, H, H, C, dev=gpu), rnd(N, H, H, C, dev=gpu)
    mean, mean2 = torch.randn(C, device=gpu) * 0.1, torch.randn(C, device=gpu) * 0.1
    istd, istd2 = torch.rand(C, device=gpu) + 0.5, torch.rand(C, device=gpu) + 0.5
    bits = torch.randint(0, 256, (N * H * H * C // 8,), device=gpu, dtype=torch.uint8)
    outs = []
    try:
        for knobs in ({}, {"epi_depth_bnr2": 4}):
            for k, v in knobs.items():
                ops.set_knob(k, v)
            r = ops.conv_dgrad_bnr(dy, w, H, H, 1, 0, res, None, xb, mean, istd, x2, mean2, istd2, None, None, None, bits)
            outs.append([t.clone() for t in r])
            ops.set_knob("epi_depth_bnr2", 2)
    finally:
        ops.set_knob("epi_depth_bnr2", 2)
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0])
        for pa, pb in zip(o[1:], outs[0][1:]):
            torch.testing.assert_close(pa.double().sum(0), pb.double().sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,k", [(1, 1000, 1), (256, 1000, 1), (64, 10, 5), (37, 1000, 8), (5, 3, 3)])
def test_topk_rows_vs_stable_sort(gpu, dtype, B, C, k):
    g = torch.Generator(device=gpu).manual_seed(B * 7 + C + k)
    x = torch.randn(B, C + 8, device=gpu, generator=g).to(dtype)[:, :C]   # row stride C+8 (padded logits)
    x[0, C // 2] = x[0].max() if B > 1 else x[0, C // 2]                   # a tie: the smaller index wins
    v, i = _ops().topk_rows(x, k, True)
    vr, ir = ref.topk_rows(x, k, True)
    assert torch.equal(i.cpu(), ir.cpu())
    assert torch.equal(v.cpu(), vr.cpu())
    (i1,) = _ops().topk_rows(x, 1, False)
    assert torch.equal(i1.view(-1).cpu(), x.float().argmax(1).cpu())


def test_topk_rows_nan_ranks_first(gpu):
    x = torch.randn(2, 100, device=gpu)
    x[1, 17] = float("nan")
    (i,) = _ops().topk_rows(x, 1, False)
    assert i.view(-1).tolist() == [int(x[0].argmax()), 17]


def test_synth_images_vs_reference(gpu):
    from pcmp.data.synthetic import SyntheticImages
    ds = SyntheticImages(n=100, image_size=32, seed=3, device=gpu)
    lab = torch.tensor([0, 4, 9, 4], device=gpu)
    col = ds.color.view(10, 3).contiguous().to(gpu)
    fr = ds.freq.contiguous().to(gpu)
    out = _ops().synth_images(lab, col, fr, 32, 12345, 0.15)
    outr = ref.synth_images(lab, col, fr, 32, 12345, 0.15)
    close(out, outr, 0, 1e-5)
    x, y = ds.get_batch(list(range(8)))
    assert x.shape == (8, 3, 32, 32) and x.dtype == torch.float32 and x.is_cuda
    assert 0.0 <= float(x.min()) and float(x.max()) <= 1.0
    assert torch.equal(y.cpu(), ds.labels(torch.arange(8)))
    x2, _ = ds.get_batch(list(range(8)))
    assert torch.equal(x, x2)          # deterministic per (seed, index window)


def _with_knob(name, value, fn):
    old = _ops().set_knob(name, value)
    try:
        return fn()
    finally:
        _ops().set_knob(name, old)


@pytest.mark.parametrize("case", ["l1_3x3", "stem_s2d"])
@pytest.mark.parametrize("epi", ["stats", "plain", "resid_relu"])
def test_halo_conv_fwd_matches_igemm_and_reference(gpu, case, epi):
    """halo_conv_kernel (stride-1 narrow-channel direct conv) == the implicit-GEMM kernel bitwise
    (same K32 chunks in the same order), and close to the fp32 reference; BN statistics partials
    (per 224-pixel tile instead of per 128) sum to the same column totals."""
    if case == "l1_3x3":
        N, H, C, R, pad = 20, 56, 64, 3, 1      # 20 * 56/4 = 280 tiles >= 256
    else:
        N, H, C, R, pad = 5, 115, 16, 4, 0      # space-to-depth stem: 115 -> 112, 5 * 56 = 280 tiles
    x = rnd(N, H, H, C, dev=gpu)
    w = rnd(64, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
    stats = epi == "stats"   # stats / plain: the overlapped-output variant; resid_relu: shared epilogue
    res = rnd(N, H + 2 * pad - R + 1, H + 2 * pad - R + 1, 64, dev=gpu) if epi == "resid_relu" else None
    run = lambda: _ops().conv_fwd(x, w, 1, pad, None, res, epi == "resid_relu", stats)
    got = _with_knob("halo", 1, run)
    base = _with_knob("halo", 0, run)
    assert torch.equal(got[0], base[0])
    yr = ref.conv_fwd(x, w, 1, pad, None, res, epi == "resid_relu", stats)
    close(got[0], yr[0])
    if stats:
        assert got[1].shape[0] == N * (H + 2 * pad - R + 1) ** 2 // 224   # one partial row per halo tile
        close(got[1].sum(0), base[1].sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("bnr", [True, False])
def test_halo_conv_dgrad_matches_igemm(gpu, bnr):
    """Layer-1 3x3 DGRAD on the halo kernel (tap-mirrored transposed weights, pad' = R-1-pad) ==
    the implicit-GEMM DGRAD bitwise, with and without the fused BN-backward reduction."""
    N, H, C = 20, 56, 64
    dy = rnd(N, H, H, C, dev=gpu)
    w = rnd(C, 3, 3, C, dev=gpu, scale=(2.0 / (9 * C)) ** 0.5)
    x = rnd(N, H, H, C, dev=gpu)
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
    if bnr:
        run = lambda: _ops().conv_dgrad_bnr(dy, w, H, H, 1, 1, None, None, x, mean, invstd, None, None, None, sc, sh)
    else:
        run = lambda: [_ops().conv_dgrad(dy, w, H, H, 1, 1, None)]
    base = _with_knob("halo", 0, run)
    # halo=4: only the overlapped BN-backward form (mask from x, no residual); halo=3 with and
    # without the overlapped output path: every DGRAD variant
    for knobs in ({"halo": 4}, {"halo": 3}, {"halo": 3, "halo_ovl": 0}):
        olds = {k: _ops().set_knob(k, v) for k, v in knobs.items()}
        try:
            got = run()
        finally:
            for k, v in olds.items():
                _ops().set_knob(k, v)
        assert torch.equal(got[0], base[0]), knobs
        if bnr:
            close(got[1].sum(0), base[1].sum(0), rtol=1e-4, atol=1e-2)
    if bnr:
        assert got[1].shape[0] == N * H * H // 224
        close(got[1].sum(0), base[1].sum(0), rtol=1e-4, atol=1e-2)
        outr = ref.conv_dgrad_bnr(dy, w, H, H, 1, 1, None, None, x, mean, invstd, None, None, None, sc, sh)
        close(got[0], outr[0])
    else:
        close(got[0], ref.conv_dgrad(dy, w, H, H, 1, 1, None))


@pytest.mark.parametrize("hw,out", [((375, 500), (224, 224)), ((224, 224), (224, 224)), ((100, 77), (224, 224)),
                                    ((1000, 333), (224, 160)), ((31, 900), (256, 256))])
def test_resize_image_matches_pil_bit_exact(gpu, hw, out):
    """Device bilinear resize (the reference's per-image Resize((224,224)) + ToTensor)
    is bit-identical to PIL.Image.resize(BILINEAR) for downscales, upscales and the identity; the
    fused NHWC bf16 / fp32 model-input forms equal the same values scaled and normalised."""
    g = torch.Generator().manual_seed(hw[0] * 7 + hw[1])
    x = torch.randint(0, 256, (2, hw[0], hw[1], 3), dtype=torch.uint8, generator=g)
    xd = x.to(gpu)
    y = _ops().resize_image(xd, out[0], out[1], 0, 0, 1.0, None, None)
    yr = ref.resize_image(x, out[0], out[1], 0, 0, 1.0)
    assert y.shape == (2, 3, out[0], out[1])
    assert torch.equal(y.cpu(), yr.cpu()), (y.int() - yr.to(gpu).int()).abs().max().item()
    mean = torch.tensor([0.485, 0.456, 0.406], device=gpu)
    std = torch.tensor([0.229, 0.224, 0.225], device=gpu)
    for mode, dt in ((1, torch.bfloat16), (2, torch.float32)):
        z = _ops().resize_image(xd, out[0], out[1], mode, 8, 1 / 255.0, mean, std)
        zr = ref.resize_image(x, out[0], out[1], mode, 8, 1 / 255.0, mean, std)
        assert z.dtype == dt and z.shape == (2, out[0], out[1], 8)
        close(z.cpu(), zr.cpu(), 1e-6, 1e-6)


def _fold_operands(gpu, N, H, K, seed):
    """g (masked BN-input gradient), x (BN input) and bn_bwd_finalize-style coefficients [3, K]."""
    torch.manual_seed(seed)
    g = rnd(N, H, H, K, dev=gpu)
    x = rnd(N, H, H, K, dev=gpu, scale=2.0) + 0.5
    coef = torch.stack([torch.rand(K, device=gpu) + 0.5, torch.randn(K, device=gpu) * 0.05,
                        torch.randn(K, device=gpu) * 0.1]).contiguous()
    return g, x, coef


@pytest.mark.parametrize("K,C,two", [(256, 64, False), (64, 256, False), (128, 512, True), (512, 128, False)])
def test_dgrad_bnr_fold(gpu, K, C, two):
    """BatchNorm-backward fold in the register-staged DGRAD: conv_dgrad_bnr(g, ..., fold_x=x,
    fold_coef=coef) == conv_dgrad_bnr(bn_bwd_apply(g, x, coef), ...): the same bf16 operand dz is
    formed while staging, so the masked gradient matches the unfolded path and the reference (1x1,
    stride 1, odd row count for the tail tile)."""
    ops = _ops()
    N, H = 3, 29
    g, x, coef = _fold_operands(gpu, N, H, K, 11)
    w = rnd(K, 1, 1, C, dev=gpu, scale=(2.0 / K) ** 0.5)
    xb, res = rnd(N, H, H, C, dev=gpu), rnd(N, H, H, C, dev=gpu)
    mean, istd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    x2 = mean2 = istd2 = None
    if two:
        x2, mean2, istd2 = rnd(N, H, H, C, dev=gpu), torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    bits = torch.randint(0, 256, (N * H * H * C // 8,), device=gpu, dtype=torch.uint8)
    dz = ops.bn_bwd_apply(g, None, x, coef, None, None, False)[0]
    close_el(dz, ref.fold_dz(g, x, coef), rel=1e-2, abs_frac=1e-3)   # fma contraction: 1-ulp bf16 differences
    args = (w, H, H, 1, 0, res, None, xb, mean, istd, x2, mean2, istd2, None, None, None, bits)
    rf = ops.conv_dgrad_bnr(g, *args, x, coef)
    ru = ops.conv_dgrad_bnr(dz, *args)
    rr = ref.conv_dgrad_bnr(g, *args, x, coef)
    close_el(rf[0], ru[0])
    close(rf[0], rr[0])
    for pf, pu in zip(rf[1:], ru[1:]):
        torch.testing.assert_close(pf.double().sum(0), pu.double().sum(0), rtol=2e-3, atol=2e-1)
    rf2 = ops.conv_dgrad_bnr(g, *args, x, coef)
    assert torch.equal(rf[0], rf2[0])


@pytest.mark.parametrize("K,C", [(256, 64), (64, 256), (512, 128), (1024, 256)])
def test_wgrad_fold(gpu, K, C):
    """BatchNorm-backward fold in the WGRAD: conv_wgrad(g, x_in, ..., fold_x=x, fold_coef=coef) ==
    conv_wgrad(bn_bwd_apply(g, x, coef), x_in, ...) (split-K and accumulate paths)."""
    ops = _ops()
    N, H = 8, 29
    g, x, coef = _fold_operands(gpu, N, H, K, 12)
    xin = rnd(N, H, H, C, dev=gpu)
    dz = ops.bn_bwd_apply(g, None, x, coef, None, None, False)[0]
    of = torch.empty(K, 1, 1, C, device=gpu)
    ou = torch.empty_like(of)
    orr = torch.empty_like(of)
    ops.conv_wgrad(g, xin, of, 1, 1, 1, 0, False, x, coef)
    ops.conv_wgrad(dz, xin, ou, 1, 1, 1, 0, False)
    ref.conv_wgrad(g, xin, orr, 1, 1, 1, 0, False, x, coef)
    close_el(of, ou, rel=1e-3, abs_frac=1e-4)
    close(of, orr, rtol=1e-2, atol=1e-2)
    ops.conv_wgrad(g, xin, of, 1, 1, 1, 0, True, x, coef)
    close(of, 2 * ou, rtol=1e-2, atol=2e-2)


def test_wgrad_fold_stem_tile(gpu):
    """Folded WGRAD of the space-to-depth stem geometry (64 filters x 4x4 taps x 16 channels: the
    64x256 tile) == WGRAD on the applied dz, and == the reference."""
    ops = _ops()
    N, P = 4, 28
    g, x, coef = _fold_operands(gpu, N, P, 64, 13)
    xin = rnd(N, P + 3, P + 3, 16, dev=gpu)
    dz = ops.bn_bwd_apply(g, None, x, coef, None, None, False)[0]
    of = torch.empty(64, 4, 4, 16, device=gpu)
    ou, orr = torch.empty_like(of), torch.empty_like(of)
    ops.conv_wgrad(g, xin, of, 4, 4, 1, 0, False, x, coef)
    ops.conv_wgrad(dz, xin, ou, 4, 4, 1, 0, False)
    ref.conv_wgrad(g, xin, orr, 4, 4, 1, 0, False, x, coef)
    close_el(of, ou, rel=1e-3, abs_frac=1e-4)
    close(of, orr, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("C,K", [(64, 256), (128, 512), (128, 64)])
def test_conv_fwd_act_fold(gpu, C, K):
    """BatchNorm-forward fold: conv_fwd(z, ..., in_scale, in_shift) == conv_fwd(bn_apply(z, relu)):
    the same bf16 operand relu(scale*z + shift) is formed while staging; BN statistics too."""
    torch.manual_seed(21)
    ops = _ops()
    N, H = 3, 29
    z = rnd(N, H, H, C, dev=gpu, scale=2.0)
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.5
    w = rnd(K, 1, 1, C, dev=gpu, scale=(2.0 / C) ** 0.5)
    y = ops.bn_apply(z, sc, sh, None, None, None, True)
    close_el(y, ref.fold_act(z, sc, sh), rel=1e-2, abs_frac=1e-3)
    rf = ops.conv_fwd(z, w, 1, 0, None, None, False, True, sc, sh)
    ru = ops.conv_fwd(y, w, 1, 0, None, None, False, True)
    rr = ref.conv_fwd(z, w, 1, 0, None, None, False, True, sc, sh)
    close_el(rf[0], ru[0])
    close(rf[0], rr[0])
    torch.testing.assert_close(rf[1].double().sum(0), ru[1].double().sum(0), rtol=2e-3, atol=5e-1)


@pytest.mark.parametrize("dzfold", [False, True])
@pytest.mark.parametrize("K,C", [(256, 64), (512, 128)])
def test_wgrad_act_fold(gpu, K, C, dzfold):
    """WGRAD with the x operand folded (relu(scale*z + shift)), alone and together with the dz fold of
    the dy operand == WGRAD on the materialised operands."""
    ops = _ops()
    N, H = 8, 29
    g, x, coef = _fold_operands(gpu, N, H, K, 14)
    z = rnd(N, H, H, C, dev=gpu, scale=2.0)
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.5
    y = ops.bn_apply(z, sc, sh, None, None, None, True)
    dz = ops.bn_bwd_apply(g, None, x, coef, None, None, False)[0]
    of = torch.empty(K, 1, 1, C, device=gpu)
    ou = torch.empty_like(of)
    if dzfold:
        ops.conv_wgrad(g, z, of, 1, 1, 1, 0, False, x, coef, sc, sh)
    else:
        ops.conv_wgrad(dz, z, of, 1, 1, 1, 0, False, None, None, sc, sh)
    ops.conv_wgrad(dz, y, ou, 1, 1, 1, 0, False)
    close_el(of, ou, rel=1e-3, abs_frac=1e-4)


@pytest.mark.parametrize("two", [False, True])
def test_dgrad_bnr_sub_sampled_residual(gpu, two):
    """conv_dgrad_bnr with a compact 1x1 stride-2 downsample DGRAD as the residual (resid_sub: added at
    the even pixels only) == the same call with that residual expanded dense (zeros elsewhere),
    bitwise, including the fused BN-backward partial sums; the compact residual itself is the
    stride-1 DGRAD of the downsample gradient on the half-resolution grid."""
    torch.manual_seed(11)
    ops = _ops()
    N, H, C, K, Kd = 8, 28, 256, 128, 512
    dh = rnd(N, H, H, K, dev=gpu)
    w = rnd(K, 1, 1, C, dev=gpu, scale=0.1)
    dcd = rnd(N, H // 2, H // 2, Kd, dev=gpu)
    wd = rnd(Kd, 1, 1, C, dev=gpu, scale=0.05)
    t_dense = ops.conv_dgrad(dcd, wd, H, H, 2, 0, None)
    t_sub = ops.conv_dgrad(dcd, wd, H // 2, H // 2, 1, 0, None)
    assert torch.equal(ref.expand_sub_resid(t_sub, H, H), t_dense)
    x = rnd(N, H, H, C, dev=gpu)
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    ymask = rnd(N, H, H, C, dev=gpu).relu()
    extra = (x, mean, invstd) if two else (None, None, None)
    a = ops.conv_dgrad_bnr(dh, w, H, H, 1, 0, t_dense, ymask, x, mean, invstd, *extra, None, None)
    b = ops.conv_dgrad_bnr(dh, w, H, H, 1, 0, t_sub, ymask, x, mean, invstd, *extra, None, None, None, None,
                           None, None, True)
    assert len(a) == len(b)
    for ta, tb in zip(a, b):
        assert torch.equal(ta, tb)
    r = ref.conv_dgrad_bnr(dh, w, H, H, 1, 0, t_sub, ymask, x, mean, invstd, *extra, resid_sub=True)
    close(b[0], r[0])
