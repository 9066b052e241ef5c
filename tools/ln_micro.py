"""Time LayerNorm fwd/bwd (BERT-base shapes, M=4096 tokens, D=768) on the HIP kernels."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

_lib.load()
ops = torch.ops.pcmp
dev = torch.device("cuda")
M, D = 4096, 768
x = torch.randn(M, D, device=dev).to(torch.bfloat16)
r = torch.randn(M, D, device=dev).to(torch.bfloat16)
g, b = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev)
y, xs, mean, rstd = ops.layernorm_fwd(x, r, g, b, 1e-12)
dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
dg, db = torch.empty(D, device=dev), torch.empty(D, device=dev)


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


print(f"blocks={torch.ops.pcmp.set_knob('ln_blocks', torch.ops.pcmp.set_knob('ln_blocks', 0))} fwd {bench(lambda: ops.layernorm_fwd(x, r, g, b, 1e-12)):.1f} us  "
      f"bwd {bench(lambda: ops.layernorm_bwd(dy, xs, mean, rstd, g, dg, db, False)):.1f} us")
