"""One fp32 conv shape of the TL forward (B=64) for PMC passes: rocprofv3 --pmc ... -- python
tools/f32_pmc.py.  SHAPE = l2_3x3 (default) | l3_3x3 | l1_1x1_256to64 | l3_1x1; MODE = fwd | dgrad |
wgrad; REPS launches after one warm-up; prints event-timed us per call and TF/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
ops = torch.ops.pcmp
SHAPES = {  # N, H, W, Cin, Cout, R, stride, pad
    "l2_3x3": (64, 28, 28, 128, 128, 3, 1, 1),
    "l3_3x3": (64, 14, 14, 256, 256, 3, 1, 1),
    "l1_1x1_256to64": (64, 56, 56, 256, 64, 1, 1, 0),
    "l3_1x1": (64, 14, 14, 1024, 256, 1, 1, 0),
}
name = os.environ.get("SHAPE", "l2_3x3")
mode = os.environ.get("MODE", "fwd")
REPS = int(os.environ.get("REPS", "10"))
N, H, W, C, K, R, s, p = SHAPES[name]
P = (H + 2 * p - R) // s + 1
dev = torch.device("cuda")
torch.manual_seed(0)
x = torch.randn(N, H, W, C, device=dev)
w = torch.randn(K, R, R, C, device=dev) * 0.05
dy = torch.randn(N, P, P, K, device=dev)
out = torch.empty(K, R, R, C, device=dev)
run = {"fwd": lambda: ops.conv_fwd(x, w, s, p, None, None, False, True),
       "dgrad": lambda: ops.conv_dgrad(dy, w, H, W, s, p, None),
       "wgrad": lambda: ops.conv_wgrad(dy, x, out, R, R, s, p, False)}[mode]
run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(REPS):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / REPS * 1e3
print(f"{name} {mode}: {us:.1f} us/call, {2.0 * N * P * P * K * R * R * C / us / 1e6:.0f} TF/s")
