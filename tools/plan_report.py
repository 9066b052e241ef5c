"""Every planner candidate's time for the batch-1 ResNet-50 convolutions (torch.ops.pcmp.plan_candidates):
kernel kind x K-split, microseconds per conv (incl. the split-K epilogue pass)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load()
ops = torch.ops.pcmp
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
for (H, C, K, R, s) in [(14, 256, 256, 3, 1), (7, 512, 512, 3, 1), (7, 2048, 512, 1, 1), (14, 1024, 256, 1, 1),
                        (28, 128, 128, 3, 1), (1, 2048, 1000, 1, 1)]:
    p = R // 2
    x = torch.randn(1, H, H, C, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(K, device=dev, generator=g)
    res = ops.plan_candidates(x, w, s, p, b, None, True)
    rows = sorted(((float(r.split()[1][:-2]), r.split()[0]) for r in res))
    print(f"{H}x{H} {C}->{K} {R}x{R}/s{s}: " + ", ".join(f"{k} {us:.1f}" for us, k in rows[:8]), flush=True)
