"""Round-6 WGRAD kernel (wgrad_dma32_kernel: LDS-DMA operands, pixel-major / image-minor reduction
order, 32x32x16 MFMAs) against the PyTorch fp32 reference ``ops/ref.conv_wgrad``
(``torch.nn.grad.conv2d_weight``) and against the register-staged kernel it replaces (knob
``wgrad_dma32`` = 0), element-wise, on every ResNet-50 WGRAD class (1x1, 3x3, strided 3x3, strided 1x1
downsample, narrow / wide Cout / Cin) plus a BERT Linear shape, over the unsplit, split-K and
accumulate paths; bitwise run-to-run determinism.  Reference: SURVEY.md §2.4.1 (conv bwd-weight),
/root/reference/pytorch_training_inference_on_image.ipynb:454-635.
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


def close_el(a, b, rel=1e-2, abs_frac=4e-3):
    a, b = a.float(), b.float()
    lim = rel * b.abs() + abs_frac * b.abs().max()
    bad = (a - b).abs() > lim
    nbad = int(bad.sum().item())
    assert nbad == 0, f"{nbad} elements outside the element-wise bound (worst {((a - b).abs() - lim).max().item():.3g})"


class _Knobs:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: _ops().set_knob(k, v) for k, v in self.kv.items()}

    def __exit__(self, *a):
        for k, v in self.old.items():
            _ops().set_knob(k, v)


# N, H, W, C, K, R, stride, pad  (N a multiple of 64: the kernel's eligibility)
SHAPES = [
    (64, 56, 56, 64, 64, 3, 1, 1),      # layer1 3x3 (BM = 64)
    (64, 56, 56, 64, 256, 1, 1, 0),     # layer1 1x1 64 -> 256 (BN = 64)
    (64, 56, 56, 256, 64, 1, 1, 0),     # layer1 1x1 256 -> 64
    (64, 56, 56, 128, 128, 3, 2, 1),    # layer2.0 3x3 stride 2
    (64, 56, 56, 256, 512, 1, 2, 0),    # layer2.0 downsample 1x1 stride 2
    (64, 14, 14, 256, 256, 3, 1, 1),    # layer3 3x3
    (128, 7, 7, 512, 512, 3, 1, 1),     # layer4 3x3 (pad taps out of the 7x7 image)
    (64, 7, 7, 2048, 512, 1, 1, 0),     # layer4 1x1 2048 -> 512 (gn = 2048)
    (4096, 1, 1, 768, 3072, 1, 1, 0),   # BERT FFN1 Linear WGRAD (tokens as the batch)
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_wgrad_dma32_matches_reference(gpu, shape):
    N, H, W, C, K, R, s, p = shape
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    torch.manual_seed(0)
    dy = rnd(N, P, Q, K, dev=gpu)
    x = rnd(N, H, W, C, dev=gpu)
    outr = torch.empty(K, R, R, C, device=gpu)
    ref.conv_wgrad(dy, x, outr, R, R, s, p, False)
    with _Knobs(wgrad_dma32=1):
        out = torch.empty_like(outr)
        _ops().conv_wgrad(dy, x, out, R, R, s, p, False)
        close_el(out, outr)
        again = torch.empty_like(outr)
        _ops().conv_wgrad(dy, x, again, R, R, s, p, False)
        assert torch.equal(out, again), "wgrad_dma32: not run-to-run deterministic"
        acc = outr.clone()
        _ops().conv_wgrad(dy, x, acc, R, R, s, p, True)
        close_el(acc, 2 * outr)
    with _Knobs(wgrad_dma32=0):
        old = torch.empty_like(outr)
        _ops().conv_wgrad(dy, x, old, R, R, s, p, False)
    close_el(out, old)


@pytest.mark.parametrize("nsplit_target", [64, 256, 1024, 4096])
def test_wgrad_dma32_split_counts(gpu, nsplit_target):
    """Every split count (1 to many K-tiles per split, a short last split) sums the whole reduction:
    the side-stream workgroup target (knob wgrad_wgs) pins the split count."""
    N, H, W, C, K = 64, 28, 28, 128, 128
    torch.manual_seed(1)
    dy = rnd(N, H, W, K, dev=gpu)
    x = rnd(N, H, W, C, dev=gpu)
    outr = torch.empty(K, 3, 3, C, device=gpu)
    ref.conv_wgrad(dy, x, outr, 3, 3, 1, 1, False)
    with _Knobs(wgrad_dma32=1, wgrad_wgs=nsplit_target):
        out = torch.empty_like(outr)
        _ops().conv_wgrad(dy, x, out, 3, 3, 1, 1, False)
    close_el(out, outr)


def test_wgrad_dma32_ineligible_falls_back(gpu):
    """N % 64 != 0 and C % 64 != 0 (stem) stay on the register-staged kernel and still match."""
    for (N, H, C, K, R, s, p) in [(48, 14, 256, 256, 3, 1, 1), (64, 115, 16, 64, 4, 1, 0)]:
        P = (H + 2 * p - R) // s + 1
        dy = rnd(N, P, P, K, dev=gpu)
        x = rnd(N, H, H, C, dev=gpu)
        outr = torch.empty(K, R, R, C, device=gpu)
        ref.conv_wgrad(dy, x, outr, R, R, s, p, False)
        out = torch.empty_like(outr)
        with _Knobs(wgrad_dma32=1):
            _ops().conv_wgrad(dy, x, out, R, R, s, p, False)
        close_el(out, outr)
