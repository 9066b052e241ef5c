"""Round-6 streaming DGRAD + BatchNorm-backward-reduce kernel (bnr_stream_kernel, knob ``bnr_stream``)
against the PyTorch fp32 reference ``ops/ref.conv_dgrad_bnr`` and against the one-tile-per-workgroup
kernels it replaces (knob off), on every layer-1/2 configuration the ResNet-50 backward sends it:
BatchNorm-backward fold of the dz operand, dual BN (block tail with a downsample), full and
sub-sampled (compact downsample DGRAD) residual, ReLU mask as bits or recomputed from x, K = 64 / 128
/ 256, 64 / 256 / 512 output channels; run-to-run bitwise determinism.  Reference: SURVEY.md §2.4.1
(BatchNorm2d / conv backward of the Bottleneck), pytorch_training_inference_on_image.ipynb:454-626.
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


def close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    lim = atol + rtol * b.abs().max().item()
    assert err <= lim, f"max err {err} > {lim}"


class _Knob:
    def __init__(self, name, v):
        self.name, self.v = name, v

    def __enter__(self):
        self.old = _ops().set_knob(self.name, self.v)

    def __exit__(self, *a):
        _ops().set_knob(self.name, self.old)


# name, N, H, K (dz channels = reduction), C (output channels), fold, dual, resid ('none'|'full'|'sub'), mask
CASES = [
    ("l1_conv1_dual", 4, 56, 64, 256, True, True, "full", "bits"),
    ("l1_conv1", 4, 56, 64, 256, True, False, "full", "bits"),
    ("l2b0_conv1_sub", 4, 56, 128, 512, True, False, "sub", "bits"),
    ("l1_conv3_mfx", 4, 56, 64, 256, True, False, "none", "mfx"),
    ("l2_conv1", 8, 28, 128, 512, False, False, "full", "bits"),
    ("l2_conv1_dual", 8, 28, 128, 512, False, True, "full", "bits"),
    ("l3b0_conv1_sub", 8, 28, 256, 512, False, False, "sub", "bits"),
    ("k64_c128", 8, 28, 64, 128, False, False, "full", "mfx"),
    ("k256_dual_sub", 8, 28, 256, 512, False, True, "sub", "bits"),
]


def _operands(gpu, N, H, K, C, fold, dual, resid, mask, seed):
    torch.manual_seed(seed)
    g = rnd(N, H, H, K, dev=gpu)
    fx = coef = None
    if fold:
        fx = rnd(N, H, H, K, dev=gpu, scale=2.0) + 0.5
        coef = torch.stack([torch.rand(K, device=gpu) + 0.5, torch.randn(K, device=gpu) * 0.05,
                            torch.randn(K, device=gpu) * 0.1]).contiguous()
    w = rnd(K, 1, 1, C, dev=gpu, scale=(2.0 / K) ** 0.5)
    x = rnd(N, H, H, C, dev=gpu)
    mean, istd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    x2 = mean2 = istd2 = None
    if dual:
        x2, mean2, istd2 = rnd(N, H, H, C, dev=gpu), torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    res = None
    if resid == "full":
        res = rnd(N, H, H, C, dev=gpu)
    elif resid == "sub":
        res = rnd(N, H // 2, H // 2, C, dev=gpu)
    bits = msc = msh = None
    if mask == "bits":
        bits = torch.randint(0, 256, (N * H * H * C // 8,), device=gpu, dtype=torch.uint8)
    else:
        msc, msh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
    return g, fx, coef, w, x, mean, istd, x2, mean2, istd2, res, bits, msc, msh


def _call(fn, H, ops_args, sub):
    g, fx, coef, w, x, mean, istd, x2, mean2, istd2, res, bits, msc, msh = ops_args
    return fn(g, w, H, H, 1, 0, res, None, x, mean, istd, x2, mean2, istd2, msc, msh, None, bits, fx, coef, sub)


@pytest.mark.parametrize("case", CASES, ids=lambda c: c[0])
def test_bnr_stream_matches(gpu, case):
    name, N, H, K, C, fold, dual, resid, mask = case
    a = _operands(gpu, N, H, K, C, fold, dual, resid, mask, 5)
    sub = resid == "sub"
    with _Knob("bnr_stream", 1):
        new = _call(_ops().conv_dgrad_bnr, H, a, sub)
        again = _call(_ops().conv_dgrad_bnr, H, a, sub)
    with _Knob("bnr_stream", 0):
        old = _call(_ops().conv_dgrad_bnr, H, a, sub)
    rr = _call(ref.conv_dgrad_bnr, H, a, sub)
    assert len(new) == len(old) == len(rr) == (3 if dual else 2)
    for t0, t1 in zip(new, again):
        assert torch.equal(t0, t1), "bnr_stream: not run-to-run deterministic"
    close(new[0], rr[0])
    # against the one-tile kernel: the same bf16 g up to 1-ulp rounding of a different MFMA order
    d = (new[0].float() - old[0].float()).abs()
    lim = 1e-2 * old[0].float().abs() + 1e-3 * old[0].float().abs().max()
    assert int((d > lim).sum()) == 0
    for pn, po, pr in zip(new[1:], old[1:], rr[1:]):
        sn, so, sr = pn.double().sum(0), po.double().sum(0), pr.double().sum(0)
        torch.testing.assert_close(sn, so, rtol=2e-3, atol=2e-1)
        torch.testing.assert_close(sn, sr, rtol=1e-2, atol=1.0)
    # the partial buffer is one row per workgroup group (<= 512: the one-launch finalize)
    assert new[1].shape[0] <= 512


def test_bnr_stream_workgroup_counts(gpu):
    """Any workgroup count (more groups than tiles, uneven tiles per group) gives the same sums."""
    a = _operands(gpu, 2, 28, 64, 256, True, False, "full", "bits", 9)
    outs = []
    for wgs in (2, 6, 64, 256, 1024, 8192):
        with _Knob("bnr_stream", 1), _Knob("bnr_stream_wgs", wgs):
            r = _call(_ops().conv_dgrad_bnr, 28, a, False)
        outs.append(r)
    for r in outs[1:]:
        assert torch.equal(r[0], outs[0][0])
        torch.testing.assert_close(r[1].double().sum(0), outs[0][1].double().sum(0), rtol=1e-5, atol=1e-3)


# name, N, H, K (input channels), C (output channels), act fold
FWD_CASES = [
    ("l1_conv3_fold", 4, 56, 64, 256, True),
    ("l1_down", 4, 56, 64, 256, False),
    ("l2_conv3_fold", 8, 28, 128, 512, True),
    ("k64_c128_fold", 8, 14, 64, 128, True),
]


@pytest.mark.parametrize("case", FWD_CASES, ids=lambda c: c[0])
def test_fwd_stream_matches(gpu, case):
    """Streaming 1x1 FWD + BatchNorm statistics (fwd_stream_kernel) == the one-tile kernels and the
    reference (conv + relu(scale * z + shift) fold), statistics summed over the partial rows."""
    name, N, H, K, C, fold = case
    torch.manual_seed(3)
    z = rnd(N, H, H, K, dev=gpu, scale=2.0)
    w = rnd(C, 1, 1, K, dev=gpu, scale=(2.0 / K) ** 0.5)
    sc = sh = None
    if fold:
        sc, sh = torch.rand(K, device=gpu) + 0.5, torch.randn(K, device=gpu) * 0.5
    with _Knob("fwd_stream", 1):
        new = _ops().conv_fwd(z, w, 1, 0, None, None, False, True, sc, sh)
        again = _ops().conv_fwd(z, w, 1, 0, None, None, False, True, sc, sh)
    with _Knob("fwd_stream", 0):
        old = _ops().conv_fwd(z, w, 1, 0, None, None, False, True, sc, sh)
    rr = ref.conv_fwd(z, w, 1, 0, None, None, False, True, sc, sh)
    for t0, t1 in zip(new, again):
        assert torch.equal(t0, t1), "fwd_stream: not run-to-run deterministic"
    close(new[0], rr[0])
    d = (new[0].float() - old[0].float()).abs()
    assert int((d > 1e-2 * old[0].float().abs() + 1e-3 * old[0].float().abs().max()).sum()) == 0
    torch.testing.assert_close(new[1].double().sum(0), old[1].double().sum(0), rtol=2e-3, atol=5e-1)
    torch.testing.assert_close(new[1].double().sum(0), rr[1].double().sum(0), rtol=1e-2, atol=2.0)
    assert new[1].shape[0] <= 512   # the streaming kernel ran (one statistics row per workgroup group)


@pytest.mark.parametrize("fold", [True, False])
@pytest.mark.parametrize("acc", [False, True])
def test_conv1x1_bwd_fused_matches(gpu, fold, acc):
    """conv1x1_bwd_fused (csrc/bwd_fused.h) == the reference composition (DGRAD + BN reduce with the mask
    recomputed from z, WGRAD against relu(scale * z + shift)) and == the separate HIP kernels."""
    torch.manual_seed(7)
    N, H, K, C = 4, 28, 256, 64
    g = rnd(N, H, H, K, dev=gpu)
    fx = coef = None
    if fold:
        fx = rnd(N, H, H, K, dev=gpu, scale=2.0) + 0.5
        coef = torch.stack([torch.rand(K, device=gpu) + 0.5, torch.randn(K, device=gpu) * 0.05,
                            torch.randn(K, device=gpu) * 0.1]).contiguous()
    w = rnd(K, 1, 1, C, dev=gpu, scale=(2.0 / K) ** 0.5)
    wt = w.reshape(K, C).t().contiguous().reshape(C, 1, 1, K)
    z = rnd(N, H, H, C, dev=gpu, scale=2.0)
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.5
    mean, istd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    base = torch.randn(K, 1, 1, C, device=gpu) if acc else torch.zeros(K, 1, 1, C, device=gpu)
    dw = base.clone()
    r = _ops().conv1x1_bwd_fused(g, fx, coef, wt, z, sc, sh, mean, istd, dw, acc)
    dw2 = base.clone()
    r2 = _ops().conv1x1_bwd_fused(g, fx, coef, wt, z, sc, sh, mean, istd, dw2, acc)
    assert torch.equal(r[0], r2[0]) and torch.equal(r[1], r2[1]) and torch.equal(dw, dw2), "not deterministic"
    dwr = base.clone()
    rr = ref.conv1x1_bwd_fused(g, fx, coef, wt, z, sc, sh, mean, istd, dwr, acc)
    close(r[0], rr[0])
    torch.testing.assert_close(r[1].double().sum(0), rr[1].double().sum(0), rtol=1e-2, atol=1.0)
    close(dw, dwr, rtol=1e-2, atol=1e-2)
    # the separate kernels (the path this replaces)
    dws = base.clone()
    _ops().conv_wgrad(g, z, dws, 1, 1, 1, 0, acc, fx, coef, sc, sh)
    rs = _ops().conv_dgrad_bnr(g, w, H, H, 1, 0, None, None, z, mean, istd, None, None, None, sc, sh, wt, None, fx,
                               coef)
    d = (r[0].float() - rs[0].float()).abs()
    assert int((d > 1e-2 * rs[0].float().abs() + 1e-3 * rs[0].float().abs().max()).sum()) == 0
    torch.testing.assert_close(r[1].double().sum(0), rs[1].double().sum(0), rtol=2e-3, atol=2e-1)
    close(dw, dws, rtol=2e-3, atol=2e-3)
