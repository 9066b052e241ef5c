"""Time the stem space-to-depth kernel at the ResNet-50 B=256 input ([256,3,224,224] fp32 NCHW ->
[256,115,115,16] bf16), min over rounds, achieved TB/s of input + output bytes.  (GPU)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
x = torch.rand(256, 3, 224, 224, device="cuda")
f = lambda: torch.ops.pcmp.image_to_s2d(x, 3, 1.0, None, None, False)  # noqa: E731
y = f()
best = 1e9
for _ in range(5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        f()
    e.record()
    torch.cuda.synchronize()
    best = min(best, s.elapsed_time(e) * 1e3 / 20)
nb = x.numel() * 4 + y.numel() * 2
print(f"image_to_s2d [256,3,224,224] f32 -> {list(y.shape)} bf16: {best:.1f} us, {nb / best / 1e6:.2f} TB/s")
