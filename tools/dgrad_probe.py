"""Where the time of the memory-bound 1x1 DGRAD + BN-backward-reduce kernels goes (ResNet-50 B=256
layer1 conv1 256->64 and layer2 conv1 512->128 backward): the same GEMM with the plain epilogue,
+ residual-gradient add, + fused BN-backward reduction (mask bits), and the unfused equivalent."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402


def t(fn, iters=10):
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
g = torch.Generator(device=dev).manual_seed(0)
for (H, C, K) in [(56, 256, 64), (28, 512, 128)]:
    N = 256
    dy = torch.randn(N, H, H, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, 1, 1, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    wt = w.reshape(K, C).t().contiguous().reshape(C, 1, 1, K)
    x = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    res = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    mean = torch.randn(C, device=dev, generator=g) * 0.1
    istd = torch.rand(C, device=dev, generator=g) + 0.5
    bits = torch.randint(0, 256, (N * H * H * C // 8,), device=dev, dtype=torch.uint8, generator=g)
    ymask = torch.randn(N, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    ops.set_knob("gemm_plan", 0)
    r = {
        "plain": t(lambda: ops.conv_dgrad(dy, w, H, H, 1, 0, None, wt)),
        "+resid": t(lambda: ops.conv_dgrad(dy, w, H, H, 1, 0, res, wt)),
        "bnr_bits+resid": t(lambda: ops.conv_dgrad_bnr(dy, w, H, H, 1, 0, res, None, x, mean, istd, None, None, None,
                                                       None, None, wt, bits)),
        "bnr_bits": t(lambda: ops.conv_dgrad_bnr(dy, w, H, H, 1, 0, None, None, x, mean, istd, None, None, None,
                                                 None, None, wt, bits)),
        "bnr_recompute_mask": t(lambda: ops.conv_dgrad_bnr(dy, w, H, H, 1, 0, res, None, x, mean, istd, None, None,
                                                           None, istd, mean, wt, None)),
        "unfused: dgrad+resid then bn_bwd_reduce": t(lambda: ops.bn_bwd_reduce(
            ops.conv_dgrad(dy, w, H, H, 1, 0, res, wt), ymask, x, mean, istd, None, None, None)),
        "copy 3 tensors (ref)": t(lambda: (x.clone(), res.clone(), ymask.clone())),
    }
    ops.set_knob("gemm_plan", 1)
    big = N * H * H * C * 2
    print(f"1x1 {C}->{K} dgrad at {H}^2 (dx {big / 1e6:.0f} MB): " + "; ".join(f"{k} {v:.1f}us" for k, v in r.items()))
