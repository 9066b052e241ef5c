"""Plain-GEMM kernels on v_mfma_f32_32x32x16_bf16 (plan kinds 9 = 128x128, 10 = 256x256, csrc/igemm.h
gemm32_kernel) forced through the planner, with and without split-K, against the fp32 reference:
Linear FWD (bias + residual + ReLU), FWD + GELU (u side output), DGRAD (+ residual), DGRAD through
GELU' -- the BERT sublayer GEMM forms, incl. tails that are not multiples of the tile."""
import pytest
import torch

import pcmp  # noqa: F401
from pcmp.ops import ref

pytestmark = pytest.mark.gpu


def _ops():
    from pcmp.ops import _lib
    assert _lib.load(), _lib.load_error()
    return torch.ops.pcmp


def rnd(*shape, dev, scale=1.0):
    return ((torch.rand(*shape, device=dev) * 2 - 1) * scale).to(torch.bfloat16)


def close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    assert err <= atol + rtol * b.abs().max().item(), err


class _Knobs:
    def __init__(self, **kv):
        self.kv, self.old = kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = _ops().set_knob(k, v)

    def __exit__(self, *a):
        for k, v in self.old.items():
            _ops().set_knob(k, v)


@pytest.mark.parametrize("mnk", [(4096, 768, 3072), (4096, 3072, 768), (2000, 520, 1024), (1100, 96, 128)])
@pytest.mark.parametrize("kind", [9, 10])
@pytest.mark.parametrize("ns", [1, 2])
def test_gemm32_linear_forms(gpu, mnk, kind, ns):
    torch.manual_seed(kind + ns)
    M, N, K = mnk
    ops = _ops()
    A = rnd(M, K, dev=gpu)
    W = rnd(N, K, dev=gpu, scale=K ** -0.5)
    bias = torch.randn(N, device=gpu)
    res = rnd(M, N, dev=gpu)
    dy = rnd(M, N, dev=gpu)
    u = rnd(M, K, dev=gpu)
    dres = rnd(M, K, dev=gpu)
    A4, W4 = A.view(M, 1, 1, K), W.view(N, 1, 1, K)
    with _Knobs(plan_force=kind, plan_nsplit=ns):
        y = ops.conv_fwd(A4, W4, 1, 0, bias, res.view(M, 1, 1, N), True, False)[0]
        g, uu = ops.linear_gelu_fwd(A, W, bias)
        dx = ops.conv_dgrad(dy.view(M, 1, 1, N), W4, 1, 1, 1, 0, dres.view(M, 1, 1, K))
        du = ops.linear_dgrad_gelu(dy, W, u)
    close(y, ref.conv_fwd(A4, W4, 1, 0, bias, res.view(M, 1, 1, N), True, False)[0])
    gr, ur = ref.linear_gelu_fwd(A, W, bias)
    close(uu, ur)
    close(g, gr)
    close(dx, ref.conv_dgrad(dy.view(M, 1, 1, N), W4, 1, 1, 1, 0, dres.view(M, 1, 1, K)))
    close(du, ref.linear_dgrad_gelu(dy, W, u))


def test_gemm32_is_a_plan_candidate(gpu):
    x = rnd(4096, 1, 1, 768, dev=gpu)
    w = rnd(3072, 1, 1, 768, dev=gpu, scale=0.03)
    log = _ops().plan_candidates(x, w, 1, 0, torch.randn(3072, device=gpu), None, False)
    assert any(e.startswith("m32_128x128") for e in log) and any(e.startswith("m32_256x256") for e in log), log
