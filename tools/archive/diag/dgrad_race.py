"""Diagnostic: repeatability of DGRAD + BN-backward reduction (mask from x) on a BIG_SHAPES case,
per DMA schedule knob (dma_pf2: bit 0 4-wave, bit 1 8-wave early prefetch)."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[2]))
import torch
import pcmp  # noqa: F401
from pcmp.ops import _lib, ref
_lib.load()
ops = torch.ops.pcmp
gpu = torch.device("cuda")
shape = tuple(int(v) for v in sys.argv[1].split(","))
N, H, W, C, K, R, s, p = shape
P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
torch.manual_seed(3)
rnd = lambda *sh, scale=1.0: (torch.randn(*sh, device=gpu) * scale).to(torch.bfloat16)
dy = rnd(N, P, Q, K)
wd = rnd(K, R, R, C, scale=(2.0 / (R * R * K)) ** 0.5)
xb = rnd(N, H, W, C)
mean, invstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
sc, sh = torch.randn(C, device=gpu), torch.randn(C, device=gpu) * 0.5
outr = ref.conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)[0].float()
for pf in (3, 1, 0):
    old = ops.set_knob("dma_pf2", pf)
    bad = []
    try:
        for it in range(12):
            out = ops.conv_dgrad_bnr(dy, wd, H, W, s, p, None, None, xb, mean, invstd, None, None, None, sc, sh)[0]
            torch.cuda.synchronize()
            e = (out.float() - outr).abs()
            bad.append((int((e > 0.05 + 0.02 * outr.abs()).sum()), round(float(e.max()), 3)))
    finally:
        ops.set_knob("dma_pf2", old)
    print("dma_pf2", pf, bad, flush=True)
