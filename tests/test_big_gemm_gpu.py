"""The round-4 "big" FWD/DGRAD kernel (igemm_big_kernel: 4 waves, 256 x 256 / 256 x 128 tiles, one
block per CU, fragments double-buffered over K-tile halves, one barrier per K-tile).

Its MFMAs accumulate every output element over K in the same order as the other FWD/DGRAD kernels
(K-tile by K-tile, the two 32-deep halves in order, one accumulator), so with the knob on its outputs
must be BITWISE equal to the default kernels' and match the fp32 reference; the BatchNorm partial
statistics (per 256-row tile instead of 128) are compared by their sums.
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


class _Knobs:
    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = _ops().set_knob(k, v)
        return self

    def __exit__(self, *a):
        for k, v in self.old.items():
            _ops().set_knob(k, v)


BIG_ON = dict(big=3, big_maxn=1 << 20, big_min256=1, big_min128=1, big_mink=1)

SHAPES = [
    # N, H, W, C, K, R, stride, pad
    (8, 14, 14, 256, 256, 3, 1, 1),     # layer-3 3x3 (M = 1568: not a multiple of 256)
    (4, 7, 7, 512, 512, 3, 1, 1),       # layer-4 3x3
    (4, 14, 14, 256, 256, 3, 2, 1),     # stride-2 3x3 (DGRAD as sub-pixel classes)
    (4, 14, 14, 256, 1024, 1, 1, 0),    # 1x1 expand
    (4, 14, 14, 1024, 256, 1, 1, 0),    # 1x1 reduce
    (3, 9, 9, 128, 384, 3, 1, 1),       # N = 384: partial 256-wide column tile
    (2, 28, 28, 128, 128, 3, 1, 1),     # N = 128: 256 x 128 tiles
]


@pytest.mark.parametrize("shape", SHAPES)
def test_big_kernel_bitwise_and_reference(gpu, shape):
    torch.manual_seed(0)
    N, H, W, C, K, R, s, p = shape
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    x = rnd(N, H, W, C, dev=gpu)
    w = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * C)) ** 0.5)
    dy = rnd(N, P, Q, K, dev=gpu)
    wd = rnd(K, R, R, C, dev=gpu, scale=(2.0 / (R * R * K)) ** 0.5)
    dres = rnd(N, H, W, C, dev=gpu)
    xb = rnd(N, H, W, C, dev=gpu)
    mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
    ymask = rnd(N, H, W, C, dev=gpu).relu()

    def run():
        out = {}
        y, st = _ops().conv_fwd(x, w, s, p, None, None, False, True)
        out["fwd"], out["fwd_stats"] = y, st.sum(0)
        out["dgrad"] = _ops().conv_dgrad(dy, wd, H, W, s, p, dres.clone())
        r = _ops().conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)
        out["bnr"], out["bnr_part"] = r[0], r[1].sum(0)
        r = _ops().conv_dgrad_bnr(dy, wd, H, W, s, p, dres.clone(), ymask, xb, mean, invstd, x, mean, invstd, None, None)
        out["bnr2"], out["bnr2_p1"], out["bnr2_p2"] = r[0], r[1].sum(0), r[2].sum(0)
        return out

    with _Knobs(big=0):
        base = run()
    with _Knobs(**BIG_ON):
        big = run()
    for k in ("fwd", "dgrad", "bnr", "bnr2"):
        assert torch.equal(big[k], base[k]), k
    for k in ("fwd_stats", "bnr_part", "bnr2_p1", "bnr2_p2"):
        close(big[k], base[k], rtol=1e-3, atol=1e-2)
    yr, str_ = ref.conv_fwd(x, w, s, p, None, None, False, True)
    close(big["fwd"], yr)
    close(big["fwd_stats"], str_.sum(0), rtol=2e-2, atol=5e-1)
    close(big["dgrad"], ref.conv_dgrad(dy, wd, H, W, s, p, dres))
    outr = ref.conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)
    close(big["bnr"], outr[0])
    close(big["bnr_part"], outr[1].sum(0), rtol=2e-2, atol=1.0)


@pytest.mark.parametrize("mnk", [(4096, 768, 3072), (4096, 3072, 768), (2000, 512, 1024)])
def test_big_kernel_plain_gemm_plans(gpu, mnk):
    """Plain GEMMs planned onto the big kernel (plan kinds 7 / 8, with and without split-K)."""
    M, N, K = mnk
    A = rnd(M, K, dev=gpu)
    B = rnd(N, K, dev=gpu, scale=K ** -0.5)
    bias = torch.randn(N, device=gpu)
    expect = ref.conv_fwd(A.view(M, 1, 1, K), B.view(N, 1, 1, K), 1, 0, bias, None, True)[0]
    for kind in (7, 8):
        for ns in (1, 2):
            with _Knobs(big=3, plan_force=kind, plan_nsplit=ns):
                got = _ops().conv_fwd(A.view(M, 1, 1, K), B.view(N, 1, 1, K), 1, 0, bias, None, True, False)[0]
            close(got, expect)


def test_big_kernel_default_policy(gpu):
    """Shipped policy: the 256x256 kernel runs for layer-3-sized N=256 convs only (plan log names it)."""
    x = rnd(256, 14, 14, 256, dev=gpu)
    w = rnd(256, 3, 3, 256, dev=gpu, scale=(2.0 / 2304) ** 0.5)
    with _Knobs(big=0):
        base = _ops().conv_fwd(x, w, 1, 1, None, None, False, True)[0]
    with _Knobs(big=1, big_maxn=256, big_min256=192):
        got = _ops().conv_fwd(x, w, 1, 1, None, None, False, True)[0]
    assert torch.equal(got, base)
