"""Isolated ResNet-50 B=256 WGRAD shapes for PMC passes (rocprofv3 --pmc ... -- python tools/wgrad_pmc.py).

SHAPE = l3_3x3 (default) | l2_3x3 | l4_3x3 | l1_3x3 | l2_1x1 | l3_1x1; REPS launches after one warm-up.
Prints the event-timed us per call and TF/s.  The split count is the autotuned / side-target one the
step would use (conv_wgrad picks it)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
SHAPES = {  # N, H, W, Cin, Cout, R, stride, pad
    "l1_3x3": (256, 56, 56, 64, 64, 3, 1, 1),
    "l2_3x3": (256, 28, 28, 128, 128, 3, 1, 1),
    "l3_3x3": (256, 14, 14, 256, 256, 3, 1, 1),
    "l4_3x3": (256, 7, 7, 512, 512, 3, 1, 1),
    "l2_1x1": (256, 28, 28, 128, 512, 1, 1, 0),
    "l3_1x1": (256, 14, 14, 1024, 256, 1, 1, 0),
}
name = os.environ.get("SHAPE", "l3_3x3")
REPS = int(os.environ.get("REPS", "10"))
N, H, W, C, K, R, s, p = SHAPES[name]
P = (H + 2 * p - R) // s + 1
dev = torch.device("cuda")
torch.manual_seed(0)
x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
dy = torch.randn(N, P, P, K, device=dev).to(torch.bfloat16)
out = torch.empty(K, R, R, C, device=dev)
ops.conv_wgrad(dy, x, out, R, R, s, p, False)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    ops.conv_wgrad(dy, x, out, R, R, s, p, False)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / REPS * 1e3
fl = 2.0 * N * P * P * K * R * R * C
print(f"wgrad {name}: {us:.1f} us/call, {fl / us / 1e6:.0f} TF/s", flush=True)
