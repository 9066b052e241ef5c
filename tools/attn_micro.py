"""Time fused attention fwd/bwd at BERT-base shapes (B=32, S=128, H=12, d=64), with/without dropout."""
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
B, S, H = 32, 128, 12
qkv = (torch.randn(B * S, 3 * H * 64, device=dev) * 0.5).to(torch.bfloat16)
ids = torch.randint(1, 100, (B, S), device=dev)
ids[:, 100:] = 0


def bench(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


for p in (0.0, 0.1):
    o, lse = ops.attention_fwd(qkv, ids, B, S, H, p, 7, 0)
    do = torch.randn_like(o)
    tf = bench(lambda: ops.attention_fwd(qkv, ids, B, S, H, p, 7, 0))
    tb = bench(lambda: ops.attention_bwd(do, qkv, o, lse, ids, B, S, H, p, 7, 0))
    print(f"p_drop={p}: fwd {tf:.1f} us  bwd {tb:.1f} us", flush=True)
