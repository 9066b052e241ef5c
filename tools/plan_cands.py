"""Print the planner's candidate timings (kind/split -> us per call, csrc/igemm.h plan_gemm) for
batch-1 ResNet-50 conv shapes: python tools/plan_cands.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
dev = torch.device("cuda", 0)
for (H, C, K, R, s) in [(7, 512, 512, 3, 1), (7, 2048, 512, 1, 1), (7, 512, 2048, 1, 1), (14, 256, 256, 3, 1),
                        (14, 1024, 256, 1, 1), (14, 256, 1024, 1, 1), (28, 128, 128, 3, 1), (28, 128, 512, 1, 1),
                        (56, 64, 64, 3, 1), (56, 64, 256, 1, 1)]:
    p = R // 2
    x = ((torch.rand(1, H, H, C, device=dev) * 2 - 1)).to(torch.bfloat16)
    w = ((torch.rand(K, R, R, C, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16)
    b = torch.randn(K, device=dev)
    resid = torch.rand(1, H // s, H // s, K, device=dev).to(torch.bfloat16) if R == 1 and K > C else None
    for _ in range(2):
        log = ops.plan_candidates(x, w, s, p, b, resid, True)
    ent = sorted(((float(e.split()[-1][:-2]), e.split()[0]) for e in log))
    print(f"H={H} C={C} K={K} R={R} M={H * H} gk={R * R * C}: " +
          "  ".join(f"{n} {t:.1f}" for t, n in ent[:14]), flush=True)
