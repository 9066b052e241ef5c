"""Isolated ResNet-50 layer-1 DGRAD (1x1, 64 -> 256 channels, 56x56, B=256) with the fused BN-backward
reduce epilogue into the previous block's tail (residual add, ReLU mask bits, partial sums of g and
g*xhat): the epilogue-bound shape that streams at ~3.6 TB/s where the plain BN-backward apply reaches
~6 TB/s (profiles/r4_fold_tile_ab.txt).  Runs it REPS times for a PMC pass:

  rocprofv3 --pmc FETCH_SIZE SQ_WAVES ... --kernel-trace -d gpurun_out/pmc -o run -- python tools/dgrad_pmc.py
Also prints the event-timed us per call and the bytes the shape needs (ideal traffic).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
REPS = int(os.environ.get("REPS", "5"))
fold = os.environ.get("FOLD", "0") == "1"

dev = torch.device("cuda")
torch.manual_seed(0)
N, hw, K, C = 256, 56, 64, 256
bf = torch.bfloat16
g = torch.randn(N, hw, hw, K, device=dev).to(bf)
x = (torch.randn(N, hw, hw, K, device=dev) + 0.5).to(bf)
coef = torch.stack([torch.rand(K, device=dev) + 0.5, torch.randn(K, device=dev) * 0.05,
                    torch.randn(K, device=dev) * 0.1]).contiguous()
w = (torch.randn(K, 1, 1, C, device=dev) * 0.05).to(bf)
wt = w.permute(3, 1, 2, 0).contiguous()
xb = torch.randn(N, hw, hw, C, device=dev).to(bf)
mean, istd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
res = torch.randn(N, hw, hw, C, device=dev).to(bf)
bits = torch.randint(0, 256, (N * hw * hw * C // 8,), device=dev, dtype=torch.uint8)
extra = (res, None, xb, mean, istd, None, None, None, None, None, wt, bits)
dz = ops.bn_bwd_apply(g, None, x, coef, None, None, False)[0]


def run():
    if fold:
        return ops.conv_dgrad_bnr(g, w, hw, hw, 1, 0, *extra, x, coef)
    return ops.conv_dgrad_bnr(dz, w, hw, hw, 1, 0, *extra)


run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    out = run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / REPS * 1e3
M = N * hw * hw
rd = M * K * 2 * (2 if fold else 1) + M * C * 2 * 2 + M * C // 8   # A (+x), resid, xb, mask bits
wr = M * C * 2                                                     # g out
print(f"{'fold' if fold else 'plain'} dgrad_bnr l1 conv1: {us:.1f} us/call, ideal read {rd / 1e6:.0f} MB "
      f"write {wr / 1e6:.0f} MB -> {(rd + wr) / us / 1e6:.2f} TB/s", flush=True)
print("outputs:", [tuple(t.shape) for t in (out if isinstance(out, (list, tuple)) else [out])])
