"""BERT-base Linear weight gradients (dW[N][C] = dy[M][N]^T x[M][C], M = 4096 tokens, fp32 output):
the framework's WGRAD (conv_wgrad 1x1, split-K + deterministic reduce, at the side-stream split
target) against hipBLASLt through torch.mm(..., out_dtype=float32) on the same operands.
Usage: python tools/linear_wgrad_micro.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
dev = torch.device("cuda")
M = 4096
SHAPES = [("qkv", 2304, 768), ("attn_out", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)]


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


tot = [0.0, 0.0, 0.0]
for name, N, C in SHAPES:
    dy = (torch.randn(M, N, device=dev) * 0.1).bfloat16()
    x = torch.randn(M, C, device=dev).bfloat16()
    out = torch.zeros(N, C, device=dev)
    ref = dy.float().t() @ x.float()
    res = []
    for wgs in (160, 384):
        old = ops.set_knob("wgrad_wgs", wgs)
        t = timed(lambda: ops.conv_wgrad(dy.view(M, 1, 1, N), x.view(M, 1, 1, C), out, 1, 1, 1, 0, False))
        ops.set_knob("wgrad_wgs", old)
        res.append(t)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    tb = timed(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    errb = ((torch.mm(dy.t(), x, out_dtype=torch.float32) - ref).abs().max() / ref.abs().max()).item()
    fl = 2.0 * M * N * C
    print(f"{name:9s} {N}x{C}x{M}: pcmp wgs160 {res[0]:6.1f} us ({fl / res[0] / 1e6:4.0f} TF) wgs384 {res[1]:6.1f} us | "
          f"hipBLASLt {tb:6.1f} us ({fl / tb / 1e6:4.0f} TF) | relerr {err:.1e} / {errb:.1e}", flush=True)
    tot[0] += res[0]
    tot[1] += res[1]
    tot[2] += tb
print(f"per layer: pcmp {tot[0]:.1f} / {tot[1]:.1f} us, hipBLASLt {tot[2]:.1f} us")
