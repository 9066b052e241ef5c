"""fp32 HIP path (``--dtype fp32``, the reference's precision): every fp32 kernel of csrc/f32.hip
against the PyTorch fp32 reference of the same op, at fp32 tolerances (relative error <= 1e-4 of
the output scale, except where the reference itself sums in another order over >10^5 terms)."""
import pytest
import torch

import pcmp  # noqa: F401
from pcmp.ops import ref

pytestmark = pytest.mark.gpu


def _ops():
    return torch.ops.pcmp


def rel_close(a, b, tol=1e-4):
    a, b = a.double(), b.double()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-30
    assert err <= tol * scale, f"max err {err:.3g} > {tol:g} x {scale:.3g}"


SHAPES = [
    # N, H, W, C, K, R, stride, pad
    (2, 32, 32, 8, 64, 7, 2, 3),      # stem (Cin padded to 8)
    (2, 14, 14, 64, 256, 1, 1, 0),    # 1x1 expand
    (2, 14, 14, 64, 64, 3, 1, 1),     # 3x3
    (2, 14, 14, 128, 128, 3, 2, 1),   # 3x3 stride 2
    (2, 14, 14, 256, 512, 1, 2, 0),   # 1x1 stride-2 downsample
    (3, 7, 7, 512, 512, 3, 1, 1),     # layer4 3x3
    (5, 1, 1, 2048, 16, 1, 1, 0),     # linear
    (64, 1, 1, 512, 1008, 1, 1, 0),   # linear, 1000(+pad) classes
]


F32_KNOBS = {
    "auto": {},                                   # the default plan
    "small": {"f32_big": 0},                      # 64x64 16x16x4 kernel only
    "big_nosplit": {"f32_blocks": 1},             # largest 32x32x2 tiles, no split
    "max_split": {"f32_blocks": 1 << 20},         # 64x64 32x32x2 tiles, split-K down to 8 K-steps
    "small_split": {"f32_big": 0, "f32_blocks": 1 << 20},
    # wave-quantisation split on grids at or above the CU target (3 "CUs" so the small shapes split)
    "qsplit": {"f32_blocks": 3, "f32_qsplit_mink": 1, "f32_qgain": 0},
}


@pytest.fixture(params=list(F32_KNOBS))
def f32_kernel(request):
    """Every launch plan of the fp32 conv GEMMs (csrc/f32.hip plan_f32): the default, the 64x64
    16x16x4 kernel, the 32x32x2 kernel without split and with the deepest split-K (partials + the
    split epilogue) and the wave-quantisation split, on the same shapes."""
    ops = _ops()
    olds = {k: ops.set_knob(k, v) for k, v in F32_KNOBS[request.param].items()}
    yield request.param
    for k, v in olds.items():
        ops.set_knob(k, v)


@pytest.mark.parametrize("shape", SHAPES + [
    (16, 28, 28, 64, 64, 3, 1, 1),     # large grid (the default policy picks the 128x128 kernel)
    (9, 15, 15, 48, 80, 3, 2, 1),      # M / N tails, stride 2, C % 16 == 0, K % 16 == 0
    (7, 9, 9, 20, 36, 3, 1, 1),        # C % 16 != 0 and K % 16 != 0: FWD/DGRAD fall back, WGRAD big
    (4, 23, 23, 16, 64, 4, 1, 0),      # s2d stem (C = 16: two taps per 32-deep K-step)
    (6, 12, 12, 16, 48, 3, 1, 1),      # C = K = 16, 3x3: gk = 144 (a half K-step tail)
])
def test_conv_fwd_dgrad_wgrad_f32(gpu, shape, f32_kernel):
    torch.manual_seed(0)
    N, H, W, C, K, R, s, p = shape
    x = torch.randn(N, H, W, C, device=gpu)
    w = torch.randn(K, R, R, C, device=gpu) * (2.0 / (R * R * C)) ** 0.5
    bias = torch.randn(K, device=gpu)
    y, st = _ops().conv_fwd(x, w, s, p, None, None, False, True)
    yr, str_ = ref.conv_fwd(x, w, s, p, None, None, False, True)
    assert y.dtype == torch.float32
    rel_close(y, yr)
    rel_close(st.sum(0), str_.sum(0), 1e-4)
    res = torch.randn_like(yr)
    rel_close(_ops().conv_fwd(x, w, s, p, bias, res, True, False)[0], ref.conv_fwd(x, w, s, p, bias, res, True)[0])
    dy = torch.randn_like(yr)
    rel_close(_ops().conv_dgrad(dy, w, H, W, s, p, None), ref.conv_dgrad(dy, w, H, W, s, p))
    out = torch.zeros(K, R, R, C, device=gpu)
    outr = torch.zeros_like(out)
    _ops().conv_wgrad(dy, x, out, R, R, s, p, False)
    ref.conv_wgrad(dy, x, outr, R, R, s, p, False)
    rel_close(out, outr, 2e-4)
    _ops().conv_wgrad(dy, x, out, R, R, s, p, True)   # accumulate
    rel_close(out, 2 * outr, 2e-4)


@pytest.mark.parametrize("shape", [
    (4, 14, 14, 64, 128, 3, 1, 1),     # 3x3 pad 1: the padding ring must stay zero (not relu(shift))
    (8, 28, 28, 128, 64, 1, 1, 0),     # 1x1
    (4, 15, 15, 32, 64, 3, 2, 1),      # stride 2, M tail
])
def test_conv_input_fold_f32(gpu, shape, f32_kernel):
    """conv_fwd / conv_wgrad reading relu(x * in_scale + in_shift) (the unmaterialised BN + ReLU of the
    producer) == the reference on the materialised activation, on every launch plan (the 64x64
    kernel materialises it itself)."""
    torch.manual_seed(4)
    N, H, W, C, K, R, s, p = shape
    x = torch.randn(N, H, W, C, device=gpu)
    w = torch.randn(K, R, R, C, device=gpu) * (2.0 / (R * R * C)) ** 0.5
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu)
    y, st = _ops().conv_fwd(x, w, s, p, None, None, False, True, sc, sh)
    yr, str_ = ref.conv_fwd(x, w, s, p, None, None, False, True, sc, sh)
    rel_close(y, yr)
    rel_close(st.sum(0), str_.sum(0))
    dy = torch.randn_like(yr)
    out, outr = torch.zeros(K, R, R, C, device=gpu), torch.zeros(K, R, R, C, device=gpu)
    _ops().conv_wgrad(dy, x, out, R, R, s, p, False, None, None, sc, sh)
    ref.conv_wgrad(dy, x, outr, R, R, s, p, False, None, None, sc, sh)
    rel_close(out, outr, 2e-4)


def test_conv_dgrad_bnr_f32(gpu, f32_kernel):
    torch.manual_seed(1)
    N, H, C, K = 2, 14, 64, 128
    w = torch.randn(K, 3, 3, C, device=gpu) * 0.05
    dy = torch.randn(N, H, H, K, device=gpu)
    x, res = torch.randn(N, H, H, C, device=gpu), torch.randn(N, H, H, C, device=gpu)
    mean, istd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    msc, msh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.1
    ym = torch.randn(N, H, H, C, device=gpu)
    bits = ref.pack_mask_bits(ym)
    for kw in (dict(ymask=ym), dict(bits=bits), dict(msc=msc)):
        r = _ops().conv_dgrad_bnr(dy, w, H, H, 1, 1, res, kw.get("ymask"), x, mean, istd, None, None, None,
                                  kw.get("msc"), msh if "msc" in kw else None, None, kw.get("bits"))
        rr = ref.conv_dgrad_bnr(dy, w, H, H, 1, 1, res, kw.get("ymask"), x, mean, istd, None, None, None,
                                kw.get("msc"), msh if "msc" in kw else None, None, kw.get("bits"))
        rel_close(r[0], rr[0])
        rel_close(r[1].sum(0), rr[1].sum(0), 2e-4)


def test_bn_and_pool_kernels_f32(gpu):
    torch.manual_seed(2)
    x = torch.randn(4, 17, 17, 64, device=gpu)
    x2 = torch.randn_like(x)
    rel_close(_ops().bn_partials(x).sum(0), ref.bn_partials(x).sum(0))
    sc, sf = torch.rand(64, device=gpu) + 0.5, torch.randn(64, device=gpu)
    sc2, sf2 = torch.rand(64, device=gpu) + 0.5, torch.randn(64, device=gpu)
    bits = torch.empty(x.numel() // 8, dtype=torch.uint8, device=gpu)
    y = _ops().bn_apply(x, sc, sf, x2, sc2, sf2, True, bits)
    yr = ref.bn_apply(x, sc, sf, x2, sc2, sf2, True)
    rel_close(y, yr, 1e-6)
    assert torch.equal(bits, ref.pack_mask_bits(yr))
    mean, istd = torch.randn(64, device=gpu) * 0.1, torch.rand(64, device=gpu) + 0.5
    dy = torch.randn_like(x)
    for a, b in zip(_ops().bn_bwd_reduce(dy, y, x, mean, istd, x2, mean, istd),
                    ref.bn_bwd_reduce(dy, y, x, mean, istd, x2, mean, istd)):
        rel_close(a.sum(0), b.sum(0))
    coef = torch.randn(3, 64, device=gpu)
    for a, b in zip(_ops().bn_bwd_apply(dy, y, x, coef, x2, coef, True), ref.bn_bwd_apply(dy, y, x, coef, x2, coef, True)):
        rel_close(a, b, 1e-6)
    yp, idx = _ops().maxpool_fwd(x, 3, 2, 1, True, sc, sf)
    ypr, idxr = ref.maxpool_fwd(x, 3, 2, 1, True, sc, sf)
    rel_close(yp, ypr, 1e-6)
    assert torch.equal(idx, idxr)
    dyp = torch.randn_like(yp)
    rel_close(_ops().maxpool_bwd(dyp, idx, 17, 17, 3, 2, 1), ref.maxpool_bwd(dyp, idxr, 17, 17, 3, 2, 1), 1e-6)
    r = _ops().maxpool_bwd_bnr(dyp, idx, x, mean, istd, sc, sf, 3, 2, 1)
    rr = ref.maxpool_bwd_bnr(dyp, idxr, x, mean, istd, sc, sf, 3, 2, 1)
    rel_close(r[0], rr[0], 1e-6)
    rel_close(r[1].sum(0), rr[1].sum(0))
    rel_close(_ops().gap_fwd(x), ref.gap_fwd(x), 1e-6)
    g = torch.randn(4, 64, device=gpu)
    rel_close(_ops().gap_bwd(g, 17, 17), ref.gap_bwd(g, 17, 17), 1e-6)
    d = _ops().dropout(x, 0.3, 77, 5 << 32)
    rel_close(d, ref.dropout(x, 0.3, 77, 5 << 32), 1e-6)
    rel_close(_ops().relu_bwd(dy, x), ref.relu_bwd(dy, x), 0)
    out = torch.zeros(64, device=gpu)
    _ops().colsum(x.view(-1, 64), out, False)
    rel_close(out, x.view(-1, 64).sum(0))
    img = torch.rand(2, 3, 20, 24, device=gpu)
    rel_close(_ops().nchw_to_nhwc_f32(img, 8, 1.0), ref.nchw_to_nhwc_f32(img, 8, 1.0), 0)


def test_resnet50_fp32_matches_torch_fp32(gpu):
    """A whole ResNet-50 at fp32 on the HIP kernels vs the same weights in stock torch.nn: eval
    logits within 1e-4 relative of torch fp32 (MIOpen); train-mode logits (batch statistics, the
    reference's TL mode) and full-network gradients judged against an fp64 torch run: the HIP fp32
    error is at most a small multiple of torch fp32's own error (BatchNorm's batch statistics over 16
    values in layer4 amplify any summation-order difference)."""
    import copy
    from pcmp.models import resnet
    from pcmp.models.torch_ref import TorchResNet
    from pcmp.ops import _lib, cross_entropy
    torch.manual_seed(3)
    _lib.set_precision("fp32")
    try:
        m = resnet.resnet50(10).to(gpu).train()
        tm = TorchResNet("resnet50", 10).to(gpu).train().load_from_pcmp(m)
        tm64 = copy.deepcopy(tm).double()
        x = torch.rand(4, 3, 64, 64, device=gpu)
        y = torch.randint(0, 10, (4,), device=gpu)
        m.eval(), tm.eval(), tm64.eval()
        with torch.no_grad():
            ze = m.forward_logits(x)
            assert ze.dtype == torch.float32
            rel_close(ze, tm(x), 1e-4)
        m.train(), tm.train(), tm64.train()
        z = m.forward_logits(x)
        zr = tm(x)
        z64 = tm64(x.double())

        def err(a, b):
            return (a.double() - b.double()).abs().max().item() / b.abs().max().item()
        e_hip, e_torch = err(z, z64), err(zr, z64)
        assert e_hip <= max(4 * e_torch, 1e-5), (e_hip, e_torch)
        cross_entropy(z, y).backward()
        torch.nn.functional.cross_entropy(zr, y).backward()
        torch.nn.functional.cross_entropy(z64, y).backward()
        pairs = [(m.layer1[0].conv1.weight.grad.permute(0, 3, 1, 2), tm.layer1[0].conv1.weight.grad,
                  tm64.layer1[0].conv1.weight.grad),
                 (m.stem.conv.weight.grad[..., :3].permute(0, 3, 1, 2), tm.conv1.weight.grad, tm64.conv1.weight.grad),
                 (m.layer3[2].conv2.weight.grad.permute(0, 3, 1, 2), tm.layer3[2].conv2.weight.grad,
                  tm64.layer3[2].conv2.weight.grad),
                 (m.fc.weight.grad[:10], tm.fc.weight.grad, tm64.fc.weight.grad)]
        for gh, gt, g64 in pairs:
            eh, et = err(gh, g64), err(gt, g64)
            assert eh <= max(4 * et, 1e-5), (eh, et)
    finally:
        _lib.set_precision("bf16")
