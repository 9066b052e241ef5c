"""Write-heavy short-K GEMM probe (ResNet-50 layer1 1x1 64->256 FWD at B=256, M=802,816): our
conv_fwd with / without the BN-statistics epilogue, hipBLASLt (torch.mm) and MIOpen (conv2d,
channels_last) on the same shape, and HBM write / copy ceilings for the same byte counts."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402


def t(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


_lib.load()
ops = torch.ops.pcmp
dev = torch.device("cuda")
for (C, K) in [(64, 256), (256, 64), (128, 512), (512, 128)]:
    H = 56 if C + K == 320 else 28
    N = 256
    M = N * H * H
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(K, 1, 1, C, device=dev) * 0.1).to(torch.bfloat16)
    byts = (M * C + M * K) * 2
    r = {}
    r["ours_stats"] = t(lambda: ops.conv_fwd(x, w, 1, 0, None, None, False, True))
    r["ours_plain"] = t(lambda: ops.conv_fwd(x, w, 1, 0, None, None, False, False))
    x2, w2 = x.view(M, C), w.view(K, C)
    r["hipblaslt_mm"] = t(lambda: torch.mm(x2, w2.t()))
    xc = x.permute(0, 3, 1, 2)
    wc = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    r["miopen_conv"] = t(lambda: torch.nn.functional.conv2d(xc, wc))
    out = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    r["fill_out"] = t(lambda: out.fill_(1.0))
    src = torch.empty(M * K, device=dev, dtype=torch.bfloat16)
    r["copy_out"] = t(lambda: out.view(-1).copy_(src))
    print(f"1x1 {C}->{K} @{H}^2 (M={M}, {byts / 1e6:.0f} MB in+out): " +
          ", ".join(f"{k} {v:.1f}us ({byts / v / 1e6:.2f} TB/s)" for k, v in r.items()))
